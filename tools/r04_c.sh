#!/bin/bash
# round-4 pass c: tolerance-triangulation A/B (T0 = before the standard-K path, T1 = with it),
# its parity tests on the new library, the peaked detector parity test
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
D=multi-camera_3d_pose_estimation_amd/mvpose
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/tri_tol_ab.py $D/libT0.so $D/libT1.so > $OUT/tri_ab.txt 2>&1 || { tail $OUT/tri_ab.txt; exit 1; }
cat $OUT/tri_ab.txt
timeout -k 10 600 python3 -u -m pytest tests/test_triangulate_gpu.py -q -s -p no:cacheprovider --timeout 180 --timeout-method thread -k tolerance > $OUT/pytest_tri.log 2>&1
rc=$?; grep -E "tolerance vs|100k|noise-free|passed|failed" $OUT/pytest_tri.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_rtmdet_gpu.py -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "peaked" > $OUT/pytest_det.log 2>&1
rc=$?; grep -E "frame [0-9]+:|peaked detector|passed|failed" $OUT/pytest_det.log | tail -8; [ $rc -le 1 ] || exit $rc
