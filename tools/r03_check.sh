#!/bin/bash
# round-3 status pass: GPU tests, then a same-box A/B of MVPOSE_NO_TBLOCK64, then the default bench
set -o pipefail
mkdir -p gpurun_out/r03g
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/r03g/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03g/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03g/pytest_gpu.log
bash tools/ab_env.sh MVPOSE_NO_TBLOCK64 2 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r03g/bench.json 2> gpurun_out/r03g/bench.err || exit 1
cat gpurun_out/r03g/bench.json | head -c 1500
