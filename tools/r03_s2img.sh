#!/bin/bash
# s2conv weight image A/B + parity (s2conv / conv planes tests)
set -o pipefail
OUT=gpurun_out/r03s2img; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_s2conv_gpu.py tests/test_conv_planes_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do for e in 0 1; do
  MVPOSE_S2_IMG=$e timeout -k 10 200 python3 tools/s2_bench.py 1024 20 > $OUT/s2_img$e.$r.log 2>&1 || exit 1
  echo "S2_IMG=$e: $(grep -E '^ *(64->128|32->256|64->256|128->256).*s2conv' $OUT/s2_img$e.$r.log | awk '{print $1, $2, $6}' | tr '\n' ' ')"
done; done | tee $OUT/ab.txt
