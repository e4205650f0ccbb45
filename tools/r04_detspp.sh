#!/bin/bash
# SPP 5x5 max as row then column max vs HEAD
# (libdetA): bit identity of the candidates, detector GPU tests, det_bench A/B, kernel stats.
set -o pipefail
mkdir -p gpurun_out/detspp
export TMPDIR=/tmp
D=multi-camera_3d_pose_estimation_amd/mvpose
for L in libdetA libmvpose; do
  MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/det_digest.py 8 640 || exit 1
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_rtmdet_gpu.py > gpurun_out/detspp/tests.log 2>&1 || { tail -30 gpurun_out/detspp/tests.log; exit 1; }
tail -1 gpurun_out/detspp/tests.log
for r in 1 2 3; do
  for L in libdetA libmvpose; do
    echo "$L $(MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/det_bench.py 128 10 2>&1 | grep batch)" || exit 1
  done
done
for L in libdetA libmvpose; do
  MVPOSE_LIB=$D/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/detspp/$L -o run -- python3 tools/det_bench.py 128 5 > gpurun_out/detspp/$L.prof.log 2>&1 || { tail gpurun_out/detspp/$L.prof.log; exit 1; }
  python3 tools/prof_summary.py $(find gpurun_out/detspp/$L -name '*kernel_stats.csv' | head -1) 40 > gpurun_out/detspp/$L.kernels.txt && grep -E "spp|total" gpurun_out/detspp/$L.kernels.txt
done
