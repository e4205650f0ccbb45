#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03j
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_sgd_joint_gpu.py tests/test_sgd_gpu.py tests/test_sgd_extrinsic_gpu.py -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_sgd.log 2>&1 || { tail -40 $OUT/pytest_sgd.log; exit 1; }
tail -2 $OUT/pytest_sgd.log; grep "sgd_joint" $OUT/pytest_sgd.log
timeout -k 10 300 python3 -u tools/sgd_bench.py > $OUT/sgd_bench.log 2>&1 || { tail $OUT/sgd_bench.log; exit 1; }
tail -5 $OUT/sgd_bench.log
