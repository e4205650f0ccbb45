#!/bin/bash
set -o pipefail
D=multi-camera_3d_pose_estimation_amd/mvpose
for L in libmvpose libtB; do
  MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/hrnet_digest.py 300 || exit 1
done
bash tools/kernel_ab.sh gpurun_out/tconvsplit_k 2 libmvpose.so libtB.so || exit 1
for f in gpurun_out/tconvsplit_k/*.txt; do echo "$f: $(grep -E 'tconv_kernel' $f | tr -s ' ' | head -2 | tr '\n' ' ')"; done
bash tools/ab_bench.sh libmvpose.so libtB.so 2 --no-cpu-baseline || exit 1
