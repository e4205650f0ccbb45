#!/bin/bash
# Balanced-batch rule (N >= CUs) for the crop-streaming kernels: conv-plane parity, then
# kernel-level A/B at 1,024 crops and bench A/B at 160 / 400 crops.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py > gpurun_out/cropbal2_planes.log 2>&1 || { tail -30 gpurun_out/cropbal2_planes.log; exit 1; }
tail -2 gpurun_out/cropbal2_planes.log
bash tools/kernel_ab.sh gpurun_out/cropbal2_k 2 libbase.so libmvpose.so || exit 1
echo "== 160 crops"; bash tools/ab_bench.sh libbase.so libmvpose.so 2 --no-cpu-baseline --frames 40 || exit 1
echo "== 400 crops"; bash tools/ab_bench.sh libmvpose.so libbase.so 1 --no-cpu-baseline --frames 100 || exit 1
