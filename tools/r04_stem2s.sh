#!/bin/bash
# streaming stem2: bit-identity vs the tile kernel + stem parity, then kernel-level A/B
set -o pipefail
mkdir -p gpurun_out/r04ss
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py -k "stem" > gpurun_out/r04ss/pytest.log 2>&1 || { tail -40 gpurun_out/r04ss/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04ss/pytest.log | tail -8
cp multi-camera_3d_pose_estimation_amd/mvpose/libmvpose.so multi-camera_3d_pose_estimation_amd/mvpose/libN.so
bash tools/kernel_ab.sh gpurun_out/r04ss 2 libA.so libN.so || exit 1
grep -H stem2 gpurun_out/r04ss/*.txt
