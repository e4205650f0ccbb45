#!/bin/bash
# tconv16 with the item DMA issued by one wave per SIMD (libH): plane parity, then timing vs shipped (libB)
set -o pipefail
mkdir -p gpurun_out/r04t11
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libH.so timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "16 or plane" > gpurun_out/r04t11/pytest.log 2>&1 || { tail -30 gpurun_out/r04t11/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04t11/pytest.log | tail -2
bash tools/kernel_ab.sh gpurun_out/r04t11 2 libB.so libH.so || exit 1
grep -H tconv16 gpurun_out/r04t11/*.txt
