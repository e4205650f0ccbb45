#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03t16; mkdir -p $OUT
for r in 1 2; do for e in "MVPOSE_TCONV16=0" "MVPOSE_TCONV16=1" "MVPOSE_TCONV16_DIAG=4" "MVPOSE_TCONV16_DIAG=2" "MVPOSE_TCONV16_DIAG=6"; do
  echo "$e: $(env $e timeout -k 10 120 python3 tools/plane_bench.py 20 128,16,12 256,8,6 | tr '\n' ' ')" || exit 1
done; done | tee $OUT/diag.txt
