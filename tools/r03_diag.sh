#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03d
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "" _NO_STORE _NO_DMA _NONE; do
  timeout -k 10 120 ./tools/s32_stamps$v 1024 > $OUT/s32$v.log 2>&1 || { cat $OUT/s32$v.log; exit 1; }
  echo "== s32$v"; cat $OUT/s32$v.log
done
timeout -k 10 300 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_tri.log 2>&1 || { tail -30 $OUT/pytest_tri.log; exit 1; }
tail -1 $OUT/pytest_tri.log
timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > $OUT/tri_roofline.log 2>&1 || exit 1
grep "V=2" $OUT/tri_roofline.log
