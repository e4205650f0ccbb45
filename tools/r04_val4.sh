#!/bin/bash
# tblock32s (all row DMAs on the conv2 waves) + stem2 (input DMA on the conv1 waves): full GPU
# suite, then whole-bench same-box A/B (libD before, libF after)
set -o pipefail
mkdir -p gpurun_out/r04v4
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04v4/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04v4/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04v4/pytest_gpu.log
grep -E "stem2_streaming|tblock32s_bitwise" gpurun_out/r04v4/pytest_gpu.log | head
bash tools/ab_bench.sh libD.so libF.so 3 || exit 1
