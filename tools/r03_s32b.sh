#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/s32_stamps 1024 > $OUT/s32_stamps.log 2>&1 || { cat $OUT/s32_stamps.log; exit 1; }
cat $OUT/s32_stamps.log
timeout -k 10 120 ./tools/tb64_stamps 1024 > $OUT/tb64_stamps.log 2>&1 || exit 1
head -1 $OUT/tb64_stamps.log
timeout -k 10 300 python3 -u tools/conv_bench.py 1024 20 > $OUT/conv_bench.log 2>&1 || exit 1
grep "C= 32" $OUT/conv_bench.log
MVPOSE_NO_TBLOCK32S=1 timeout -k 10 300 python3 -u tools/conv_bench.py 1024 20 > $OUT/conv_bench_tile.log 2>&1 || exit 1
grep "C= 32" $OUT/conv_bench_tile.log
