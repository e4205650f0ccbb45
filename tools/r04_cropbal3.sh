#!/bin/bash
# Balanced-batch rule (N >= CUs; tblock64 strided mode a separate template instance):
# conv-plane parity, then bench A/B at 40 / 160 / 400 / 1,024 crops.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_planes_gpu.py > gpurun_out/cropbal3_planes.log 2>&1 || { tail -30 gpurun_out/cropbal3_planes.log; exit 1; }
tail -2 gpurun_out/cropbal3_planes.log
for F in 10 40 100 256; do
  echo "== $((F * 4)) crops"; bash tools/ab_bench.sh libbase.so libmvpose.so 2 --no-cpu-baseline --frames $F || exit 1
done
