#!/bin/bash
# detector GEMM kernel without its K-step DMA after the first 3 chunks (libDN, timing only) vs shipped (libF)
set -o pipefail
mkdir -p gpurun_out/${TAG:-r04d15}
export TMPDIR=/tmp
for L in ${LIBS:-libF libDN}; do
  MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG:-r04d15}/$L -o run -- python3 tools/det_bench.py 128 3 > gpurun_out/${TAG:-r04d15}/$L.log 2>&1 || { tail gpurun_out/${TAG:-r04d15}/$L.log; exit 1; }
  grep batch gpurun_out/${TAG:-r04d15}/$L.log
  python3 tools/prof_summary.py $(find gpurun_out/${TAG:-r04d15}/$L -name '*kernel_stats.csv' | head -1) 8
done
