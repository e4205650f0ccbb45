#!/bin/bash
# tconv16 (128-cout tiles, weight image) vs tconv (64-cout tiles) on the 128/256-channel planes: parity tests + per-conv time
set -o pipefail
OUT=gpurun_out/r03t16; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_conv_planes_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "basic_block or batch_positions" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do for e in "MVPOSE_TCONV16=0" "MVPOSE_TCONV16=1" "MVPOSE_TCONV16_DIAG=2"; do
  echo "$e: $(env $e timeout -k 10 120 python3 tools/plane_bench.py 20 128,16,12 256,8,6 | tr '\n' ' ')" || exit 1
done; done | tee $OUT/planes.txt
