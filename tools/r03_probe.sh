#!/bin/bash
# probes: triangulation tests + roofline, v_rcp_f64 accuracy, tblock64 phase stamps
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03p
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_tri.log 2>&1 || { tail -40 $OUT/pytest_tri.log; exit 1; }
tail -2 $OUT/pytest_tri.log; grep "bit-identical" $OUT/pytest_tri.log
timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > $OUT/tri_roofline.log 2>&1 || exit 1
grep -h "V=2" $OUT/tri_roofline.log
timeout -k 10 60 ./tools/rcp_probe > $OUT/rcp_probe.log 2>&1 || exit 1
cat $OUT/rcp_probe.log
timeout -k 10 120 ./tools/tb64_stamps 1024 > $OUT/tb64_stamps.log 2>&1 || exit 1
cat $OUT/tb64_stamps.log
