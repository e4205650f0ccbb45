#!/bin/bash
# tblock32s conv1 row reuse (libR): bit-identity vs the tile kernel, then timing vs shipped (libG)
set -o pipefail
mkdir -p gpurun_out/r04t19
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libR.so timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "tblock32s" > gpurun_out/r04t19/pytest.log 2>&1 || { tail -30 gpurun_out/r04t19/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04t19/pytest.log | tail -7
bash tools/kernel_ab.sh gpurun_out/r04t19 2 libG.so libR.so || exit 1
grep -H tblock32s gpurun_out/r04t19/*.txt
