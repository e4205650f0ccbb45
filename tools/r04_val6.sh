#!/bin/bash
# tblock32s row reuse: full GPU suite, whole-bench same-box A/B (libG before, libR after)
set -o pipefail
mkdir -p gpurun_out/r04v6
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04v6/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04v6/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04v6/pytest_gpu.log
bash tools/ab_bench.sh libG.so libR.so 3 || exit 1
