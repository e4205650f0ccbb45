#!/bin/bash
# SGD: smoothness terms in LDS (libST), + pass B two points per round (libST2) vs shipped (libJ)
set -o pipefail
mkdir -p gpurun_out/r04o5
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libST2.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sgd_gpu.py tests/test_sgd_joint_gpu.py > gpurun_out/r04o5/pytest.log 2>&1 || { tail -30 gpurun_out/r04o5/pytest.log; exit 1; }
tail -1 gpurun_out/r04o5/pytest.log
for r in 1 2 3; do
  for L in libJ libST libST2; do
    MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 240 python3 tools/sgd_line_ab.py 2>/dev/null | tail -1
  done
done
