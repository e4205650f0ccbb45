#!/bin/bash
# Depthwise 5x5: input-row loop unrolled by 1 (HEAD) / 2 / 3: candidate digests + det_bench A/B.
set -o pipefail
D=multi-camera_3d_pose_estimation_amd/mvpose
for L in libmvpose libdw2 libdw3; do
  MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/det_digest.py 8 640 || exit 1
done
for r in 1 2; do
  for L in libmvpose libdw2 libdw3; do
    echo "$L $(MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/det_bench.py 128 10 2>&1 | grep batch)" || exit 1
  done
done
