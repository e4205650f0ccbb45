#!/bin/bash
# validation: full GPU suite, whole-bench same-box A/B (libR before, libS after), forward breakdown
set -o pipefail
mkdir -p gpurun_out/r04v7
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04v7/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04v7/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04v7/pytest_gpu.log
bash tools/ab_bench.sh libR.so libS.so 3 || exit 1
bash tools/kernel_ab.sh gpurun_out/r04v7 1 libS.so || exit 1
head -25 gpurun_out/r04v7/libS.1.txt
