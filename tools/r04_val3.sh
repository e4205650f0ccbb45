#!/bin/bash
# DMA-split kernels: full GPU suite, then whole-bench same-box A/B (libB before, libD after)
set -o pipefail
mkdir -p gpurun_out/r04v3
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04v3/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04v3/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04v3/pytest_gpu.log
bash tools/ab_bench.sh libB.so libD.so 3 || exit 1
