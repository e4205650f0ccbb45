#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03t16skip; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_conv_planes_gpu.py tests/test_backbone_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do for L in libA.so libB.so; do echo "$L $(MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L timeout -k 10 120 python3 tools/plane_bench.py 20 128,16,12 256,8,6 | tr '\n' ' ')" || exit 1; done; done | tee $OUT/plane.txt
bash tools/ab_bench.sh libA.so libB.so 3 --no-cpu-baseline | tee $OUT/ab.txt
