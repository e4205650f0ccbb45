#!/bin/bash
# detector GEMM tile configurations (env tuning switches) on one box
set -o pipefail
OUT=gpurun_out/r03detcfg; mkdir -p $OUT
for r in 1 2; do for e in "X=0" "MVPOSE_DET_PW=4" "MVPOSE_DET_FP=8" "MVPOSE_DET_RING=4" "MVPOSE_DET_BN=128"; do
  env $e timeout -k 10 200 python3 tools/det_bench.py > $OUT/det.log 2>&1 || { tail $OUT/det.log; exit 1; }
  echo "$e: $(grep -o 'batch.*' $OUT/det.log | tail -1)"
done; done | tee $OUT/cfg.txt
