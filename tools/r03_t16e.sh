#!/bin/bash
# tconv16 epilogue attribution (timing only): 2 = no epilogue, 8 = barrier only, 16 = no global stores, 32 = no staging writes
set -o pipefail
OUT=gpurun_out/r03t16; mkdir -p $OUT
for r in 1 2; do for d in 0 2 8 16 32 48; do
  echo "DIAG=$d: $(MVPOSE_TCONV16_DIAG=$d timeout -k 10 120 python3 tools/plane_bench.py 20 128,16,12 256,8,6 | tr '\n' ' ')" || exit 1
done; done | tee $OUT/epi.txt
