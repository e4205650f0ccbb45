#!/bin/bash
# (apply tools/pending/tconv_dma_split.patch and build libmvpose.so first; libtA.so = HEAD)
# tconv_kernel with one DMA-issuing wave per SIMD vs HEAD (libtA): backbone digests, conv-plane
# tests, kernel-level A/B of the 1,024-crop forward, bench A/B.
set -o pipefail
D=multi-camera_3d_pose_estimation_amd/mvpose
for L in libtA libmvpose; do
  MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/hrnet_digest.py 300 || exit 1
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py > gpurun_out/tconvsplit_planes.log 2>&1 || { tail -30 gpurun_out/tconvsplit_planes.log; exit 1; }
tail -1 gpurun_out/tconvsplit_planes.log
bash tools/kernel_ab.sh gpurun_out/tconvsplit_k 2 libtA.so libmvpose.so || exit 1
for f in gpurun_out/tconvsplit_k/*.txt; do echo "$f: $(grep -E 'tconv_kernel' $f | tr -s ' ' | head -2 | tr '\n' ' ')"; done
bash tools/ab_bench.sh libtA.so libmvpose.so 2 --no-cpu-baseline || exit 1
