#!/bin/bash
# detector GEMM weight image: parity + same-box A/B
set -o pipefail
OUT=gpurun_out/r03detimg; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_rtmdet_gpu.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do for e in 0 1; do
  MVPOSE_DET_WIMG=$e timeout -k 10 200 python3 tools/det_bench.py > $OUT/det_$e.$r.log 2>&1 || { tail $OUT/det_$e.$r.log; exit 1; }
  echo "WIMG=$e: $(tail -2 $OUT/det_$e.$r.log | tr '\n' ' ')"
done; done | tee $OUT/ab.txt
