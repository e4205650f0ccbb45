#!/bin/bash
# SGD pass B over per-joint segment lists (libJ) vs shipped (libA): SGD GPU tests, then bench's config-5 line
set -o pipefail
mkdir -p gpurun_out/r04o4
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libJ.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sgd_gpu.py tests/test_sgd_joint_gpu.py > gpurun_out/r04o4/pytest.log 2>&1 || { tail -30 gpurun_out/r04o4/pytest.log; exit 1; }
tail -1 gpurun_out/r04o4/pytest.log
for r in 1 2 3; do
  for L in libA libJ; do
    MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 240 python3 tools/sgd_line_ab.py 2>/dev/null | tail -1
  done
done
