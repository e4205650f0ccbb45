#!/bin/bash
# round-4 closing profile (tools/r04_prof.sh recipe + the forward breakdown): default bench,
# rocprofv3 kernel trace + stats of the bench, backbone forward breakdown, separate
# FETCH_SIZE / WRITE_SIZE PMC passes -> traffic json
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${TAG:-r04x}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
head -c 600 $OUT/bench.json; echo
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
python3 $ROOT/tools/prof_summary.py $(find $OUT/trace -name '*kernel_stats.csv' | head -1) 45 > $OUT/kernels.txt && head -12 $OUT/kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/fwd -o run -- python3 $ROOT/tools/prof_backbone.py 1024 3 > $OUT/fwd.log 2>&1 || { tail $OUT/fwd.log; exit 1; }
python3 $ROOT/tools/fwd_breakdown.py $(find $OUT/fwd -name '*kernel_trace.csv' | head -1) > $OUT/forward_breakdown.txt && tail -1 $OUT/forward_breakdown.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/pmc_fetch.log 2>&1 || { tail $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra > $OUT/pmc_write.log 2>&1 || { tail $OUT/pmc_write.log; exit 1; }
python3 $ROOT/tools/pmc_traffic.py $(find $OUT/pmc_fetch -name '*counter_collection.csv' | head -1) \
    $(find $OUT/pmc_write -name '*counter_collection.csv' | head -1) $OUT/traffic.json > /dev/null && head -8 $OUT/traffic.json
