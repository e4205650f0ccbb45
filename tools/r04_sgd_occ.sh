#!/bin/bash
# SGD occupancy A/B (config 5, M = 1 / 256): shipped (A), block_sum without the unrolled
# partial loads (B), 1024-thread workgroups at kU = 2 (C), kU = 1 (D), kU = 4 (E)
set -o pipefail
mkdir -p gpurun_out/r04o
for r in 1 2; do
  for L in libA libB libC libD libE; do
    MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 240 python3 tools/sgd_bench.py 200 > gpurun_out/r04o/$L.$r.log 2>&1 || { tail gpurun_out/r04o/$L.$r.log; exit 1; }
    echo "== $L $r"; cat gpurun_out/r04o/$L.$r.log
  done
done
