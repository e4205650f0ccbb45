#!/bin/bash
# same-box A/B of an env switch: bash tools/ab_env.sh VAR rounds
set -o pipefail
V=$1; R=${2:-2}
for r in $(seq 1 "$R"); do
  for e in 0 1; do
    if [ $e = 1 ]; then export $V=1; else unset $V; fi
    timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline > gpurun_out/abenv_$e.$r.log 2>&1 || exit 1
    echo "$V=$e $(grep -o '"value": [0-9.]*' gpurun_out/abenv_$e.$r.log | head -1)"
  done
done
