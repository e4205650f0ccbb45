#!/bin/bash
# stem2 4+4 role split (libQ): bit-identity vs the tile kernel, then timing vs libZ / tile (libA)
set -o pipefail
mkdir -p gpurun_out/r04st6
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libQ.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "stem" > gpurun_out/r04st6/pytest.log 2>&1 || { tail -30 gpurun_out/r04st6/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04st6/pytest.log | tail -2
bash tools/kernel_ab.sh gpurun_out/r04st6 2 libA.so libZ.so libQ.so || exit 1
grep -H stem2 gpurun_out/r04st6/*.txt
