#!/bin/bash
# detector kernel breakdown at one 512-camera-frame forward (the bench's detector line)
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/det_bench.py 512 5 > $OUT/bench.log 2>&1 && cat $OUT/bench.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/det_bench.py 512 2 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/trace -name '*kernel_stats.csv' | head -1) 30 > $OUT/kernels.txt && cat $OUT/kernels.txt
