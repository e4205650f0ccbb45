#!/bin/bash
# Detector halo tiles of 4 output rows (default) vs 2 (HEAD, libdetA): detector GPU tests
# (layer by layer vs the interpreter, 4-row vs 2-row bit identity, end to end), then a
# same-box det_bench A/B and a kernel trace of each.
set -o pipefail
mkdir -p gpurun_out/dethalo
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rtmdet_gpu.py > gpurun_out/dethalo/tests.log 2>&1 || { tail -30 gpurun_out/dethalo/tests.log; exit 1; }
tail -1 gpurun_out/dethalo/tests.log
D=multi-camera_3d_pose_estimation_amd/mvpose
for r in 1 2 3; do
  for L in libdetA libmvpose; do
    echo "$L $(MVPOSE_LIB=$D/$L.so timeout -k 10 180 python3 tools/det_bench.py 128 10 2>&1 | grep batch)" || exit 1
  done
done
for L in libdetA libmvpose; do
  MVPOSE_LIB=$D/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dethalo/$L -o run -- python3 tools/det_bench.py 128 5 > gpurun_out/dethalo/$L.prof.log 2>&1 || { tail gpurun_out/dethalo/$L.prof.log; exit 1; }
  python3 tools/prof_summary.py $(find gpurun_out/dethalo/$L -name '*kernel_stats.csv' | head -1) 12 > gpurun_out/dethalo/$L.kernels.txt && grep -E "halo|sum" gpurun_out/dethalo/$L.kernels.txt
done
