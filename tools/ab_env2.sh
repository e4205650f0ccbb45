#!/bin/bash
# same-box A/B of an environment switch with explicit values:
#   bash tools/ab_env2.sh VAR VALUE_A VALUE_B [rounds]
set -o pipefail
V=$1; A=$2; B=$3; R=${4:-2}
for r in $(seq 1 "$R"); do
  for val in "$A" "$B"; do
    env "$V=$val" timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline > gpurun_out/abenv2_$val.$r.log 2>&1 || exit 1
    echo "$V=$val $(grep -o '"value": [0-9.]*' gpurun_out/abenv2_$val.$r.log | head -1) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/abenv2_$val.$r.log | head -1)"
  done
done
