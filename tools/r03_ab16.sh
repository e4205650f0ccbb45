#!/bin/bash
# GPU suite + same-box A/B of the weight-image kernels (tconv16 + s2conv image) on the bench
set -o pipefail
OUT=gpurun_out/r03ab16; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2 3; do for e in off on; do
  if [ $e = off ]; then export MVPOSE_TCONV16=0 MVPOSE_S2_IMG=0; else unset MVPOSE_TCONV16 MVPOSE_S2_IMG; fi
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > $OUT/ab_$e.$r.log 2>&1 || exit 1
  echo "$e $(grep -o '"value": [0-9.]*' $OUT/ab_$e.$r.log | head -1) $(grep -o '"avg_launch_ms": [0-9.]*' $OUT/ab_$e.$r.log | head -1)"
done; done | tee $OUT/ab.txt
