#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03u
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_tri.log 2>&1 || { tail -30 $OUT/pytest_tri.log; exit 1; }
tail -1 $OUT/pytest_tri.log; grep "bit-identical" $OUT/pytest_tri.log
timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > $OUT/tri_roofline.log 2>&1 || exit 1
grep "V=2" $OUT/tri_roofline.log
for v in "" _pf3 _pf4; do
  timeout -k 10 120 ./tools/tb64_stamps$v 1024 > $OUT/tb64$v.log 2>&1 || { cat $OUT/tb64$v.log; exit 1; }
  echo "== tb64$v"; cat $OUT/tb64$v.log
done
