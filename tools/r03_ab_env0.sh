#!/bin/bash
# same-box bench A/B of an env switch set to 0 vs unset, after the listed tests: bash tools/r03_ab_env0.sh VAR rounds [pytest args...]
set -o pipefail
V=$1; R=$2; shift 2
OUT=gpurun_out/ab_$V; mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 400 python3 -u -m pytest "$@" -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for r in $(seq 1 "$R"); do for e in 0 1; do
  if [ $e = 0 ]; then export $V=0; else unset $V; fi
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > $OUT/b_$e.$r.log 2>&1 || exit 1
  echo "$V=$e $(grep -o '"value": [0-9.]*' $OUT/b_$e.$r.log | head -1) $(grep -o '"avg_launch_ms": [0-9.]*' $OUT/b_$e.$r.log | head -1)"
done; done | tee $OUT/ab.txt
