#!/bin/bash
# tconv 128/256 diagnostics: per-conv time with the DMA-skip / no-store switches
set -o pipefail
OUT=gpurun_out/r03t128; mkdir -p $OUT
for d in 0 14 30 46 62; do
  echo "diag=$d: $(MVPOSE_TCONV_DIAG=$d timeout -k 10 120 python3 tools/plane_bench.py 20 128,16,12 256,8,6 | tr '\n' ' ')" || exit 1
done | tee $OUT/diag.txt
