#!/bin/bash
# Balanced-batch rule for the crop-streaming kernels: parity, full suite, same-box A/B at the
# headline batch (1024 crops) and at unbalanced batches (400 / 160 crops).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py > gpurun_out/cropbal_planes.log 2>&1 || { tail -30 gpurun_out/cropbal_planes.log; exit 1; }
tail -3 gpurun_out/cropbal_planes.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/cropbal_suite.log 2>&1 || { tail -30 gpurun_out/cropbal_suite.log; exit 1; }
tail -3 gpurun_out/cropbal_suite.log
echo "== 1024 crops"; bash tools/ab_bench.sh libbase.so libmvpose.so 2 --no-cpu-baseline || exit 1
echo "== 400 crops"; bash tools/ab_bench.sh libbase.so libmvpose.so 2 --no-cpu-baseline --frames 100 || exit 1
echo "== 160 crops"; bash tools/ab_bench.sh libbase.so libmvpose.so 2 --no-cpu-baseline --frames 40 || exit 1
