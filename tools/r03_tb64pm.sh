#!/bin/bash
# tblock64 pixel-major ring: bitwise test + plane time + same-box bench A/B (libA = plane-major, libB = pixel-major)
set -o pipefail
OUT=gpurun_out/r03tb64pm; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_conv_planes_gpu.py tests/test_backbone_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for L in libA.so libB.so; do echo "$L $(MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L timeout -k 10 120 python3 tools/plane_bench.py 20 64,32,24 | tr '\n' ' ')" || exit 1; done | tee $OUT/plane.txt
bash tools/ab_bench.sh libA.so libB.so 3 --no-cpu-baseline | tee $OUT/ab.txt
