#!/bin/bash
# tblock64 reusing intermediate rows across a crop's tiles (libG): bit-identity vs two tconv
# launches, backbone parity, then kernel-level A/B vs shipped (libF)
set -o pipefail
mkdir -p gpurun_out/r04t17
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libG.so timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "tblock64" > gpurun_out/r04t17/pytest.log 2>&1 || { tail -30 gpurun_out/r04t17/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04t17/pytest.log | tail -6
bash tools/kernel_ab.sh gpurun_out/r04t17 2 libF.so libG.so || exit 1
grep -H tblock64 gpurun_out/r04t17/*.txt
