#!/bin/bash
# SGD adjoint with hardware reciprocals: SGD parity tests (libB) + sgd_bench A/B
set -o pipefail
OUT=gpurun_out/r03sgdrcp; mkdir -p $OUT
D=multi-camera_3d_pose_estimation_amd/mvpose
MVPOSE_LIB=$D/libB.so timeout -k 10 400 python3 -u -m pytest tests/test_sgd_gpu.py tests/test_sgd_joint_gpu.py tests/test_sgd_extrinsic_gpu.py -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
grep -E "passed|failed" $OUT/pytest.log | tail -1; grep -iE "dev|d traj" $OUT/pytest.log | head -12
for r in 1 2; do for L in libA.so libB.so; do
  MVPOSE_LIB=$D/$L timeout -k 10 200 python3 tools/sgd_bench.py > $OUT/sgd_$L.$r.log 2>&1 || { tail $OUT/sgd_$L.$r.log; exit 1; }
  echo "$L $(tail -3 $OUT/sgd_$L.$r.log | tr '\n' ' ' | cut -c1-400)"
done; done | tee $OUT/ab.txt
