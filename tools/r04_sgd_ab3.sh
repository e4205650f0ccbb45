#!/bin/bash
# SGD A/B on bench.py's config-5 line: shipped (A) vs variant libraries given as arguments
set -o pipefail
mkdir -p gpurun_out/r04o3
for r in 1 2 3; do
  for L in libA "$@"; do
    MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 240 python3 tools/sgd_line_ab.py > gpurun_out/r04o3/$L.$r.log 2>&1 || { tail gpurun_out/r04o3/$L.$r.log; exit 1; }
    tail -1 gpurun_out/r04o3/$L.$r.log
  done
done
