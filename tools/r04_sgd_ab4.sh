#!/bin/bash
# SGD pass A: compile-time instance of the point loop for the default settings, branch-free
# finite mask (U1), plus the camera loop unrolled by 2 (U2), vs HEAD (A); SGD GPU tests first.
set -o pipefail
mkdir -p gpurun_out/r04o6
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sgd_gpu.py tests/test_sgd_joint_gpu.py tests/test_sgd_extrinsic_gpu.py > gpurun_out/r04o6/tests.log 2>&1 || { tail -30 gpurun_out/r04o6/tests.log; exit 1; }
tail -2 gpurun_out/r04o6/tests.log
for r in 1 2 3; do
  for L in libsgdA libsgdU1 libsgdU2; do
    MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 240 python3 tools/sgd_line_ab.py > gpurun_out/r04o6/$L.$r.log 2>&1 || { tail gpurun_out/r04o6/$L.$r.log; exit 1; }
    tail -1 gpurun_out/r04o6/$L.$r.log
  done
done
