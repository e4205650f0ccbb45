#!/bin/bash
# fuse 3<-1 chain's 64->64 3x3/s2 @32x24 on s2conv (BM = 64, 2 crops per tile; libB64) vs conv_mfma_kernel (libZ0)
set -o pipefail
mkdir -p gpurun_out/r04t22
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libB64.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_s2conv_gpu.py > gpurun_out/r04t22/pytest.log 2>&1 || { tail -30 gpurun_out/r04t22/pytest.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04t22/pytest.log | tail -2
bash tools/kernel_ab.sh gpurun_out/r04t22 2 libZ0.so libB64.so || exit 1
grep -H "conv_mfma\|s2conv_kernel<64, 32, 24" gpurun_out/r04t22/*.txt
