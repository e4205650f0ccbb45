#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -m pytest tests/test_conv_planes_gpu.py -x -q -s -k "tblock32s or basic_block_vs_reference" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_s32.log 2>&1 || { tail -40 $OUT/pytest_s32.log; exit 1; }
tail -1 $OUT/pytest_s32.log
timeout -k 10 120 ./tools/s32_stamps 1024 > $OUT/s32_stamps.log 2>&1 || { cat $OUT/s32_stamps.log; exit 1; }
cat $OUT/s32_stamps.log
bash tools/ab_env.sh MVPOSE_NO_TBLOCK32S 2 || exit 1
