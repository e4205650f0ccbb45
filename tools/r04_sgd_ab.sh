#!/bin/bash
# SGD division guard: SGD parity tests on libB (the guarded tree) + sgd_bench A/B against libA
set -o pipefail
OUT=gpurun_out/r04sgd; mkdir -p $OUT
D=multi-camera_3d_pose_estimation_amd/mvpose
export TMPDIR=/tmp
MVPOSE_LIB=$D/libB.so timeout -k 10 600 python3 -u -m pytest tests/test_sgd_gpu.py tests/test_sgd_joint_gpu.py tests/test_sgd_extrinsic_gpu.py -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -8; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for L in libA.so libB.so; do
  MVPOSE_LIB=$D/$L timeout -k 10 200 python3 tools/sgd_bench.py > $OUT/sgd_$L.$r.log 2>&1 || { tail $OUT/sgd_$L.$r.log; exit 1; }
  echo "$L $(tail -2 $OUT/sgd_$L.$r.log | tr '\n' ' ' | cut -c1-300)"
done; done | tee $OUT/ab.txt
