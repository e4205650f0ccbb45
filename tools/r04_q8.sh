#!/bin/bash
# stem2 with the input DMA two strips ahead (libD2): bit-identity vs the tile kernel, timing vs shipped (libB)
set -o pipefail
mkdir -p gpurun_out/r04st8
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libD2.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "stem" > gpurun_out/r04st8/pytest.log 2>&1 || { tail -30 gpurun_out/r04st8/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04st8/pytest.log | tail -2
bash tools/kernel_ab.sh gpurun_out/r04st8 2 libB.so libD2.so || exit 1
grep -H stem2 gpurun_out/r04st8/*.txt
