#!/bin/bash
# triangulation tolerance-kernel pass: parity tests (both f32-iteration variants), roofline A/B
set -o pipefail
mkdir -p gpurun_out/r03t
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03t/pytest_tri.log 2>&1 || { tail -40 gpurun_out/r03t/pytest_tri.log; exit 1; }
tail -3 gpurun_out/r03t/pytest_tri.log
MVPOSE_TRI_F32=4 timeout -k 10 300 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -s -k tolerance -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03t/pytest_tri_f32x4.log 2>&1 || { tail -40 gpurun_out/r03t/pytest_tri_f32x4.log; exit 1; }
grep -E "bit-identical|passed|failed" gpurun_out/r03t/pytest_tri_f32x4.log
timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > gpurun_out/r03t/tri_roofline.log 2>&1 || exit 1
MVPOSE_TRI_F32=4 timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > gpurun_out/r03t/tri_roofline_f32x4.log 2>&1 || exit 1
grep -h "V=2" gpurun_out/r03t/tri_roofline*.log
