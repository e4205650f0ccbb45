#!/bin/bash
# tblock64 halo DMA split over all 4 waves, residual read at the end of the previous phase (libG2) vs row reuse (libG)
# launches, backbone parity, then kernel-level A/B vs shipped (libF)
set -o pipefail
mkdir -p gpurun_out/r04t18
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libG2.so timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "tblock64" > gpurun_out/r04t18/pytest.log 2>&1 || { tail -30 gpurun_out/r04t18/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04t18/pytest.log | tail -6
bash tools/kernel_ab.sh gpurun_out/r04t18 2 libG.so libG2.so || exit 1
grep -H tblock64 gpurun_out/r04t18/*.txt
