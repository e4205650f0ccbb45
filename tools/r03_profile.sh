#!/bin/bash
# Round-3 measurement: GPU tests, default bench (with CPU baseline), rocprofv3 kernel trace +
# stats of the bench, one backbone forward's kernel trace (breakdown), separate FETCH_SIZE and
# WRITE_SIZE passes -> traffic json.  Every GPU step has its own limit; stop at the first failure.
set -o pipefail
R=${1:-r03h}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 600 python3 -u -m pytest "$ROOT/tests" -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail "$OUT/bench.err"; exit 1; }
head -c 1200 "$OUT/bench.json"; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
python3 "$ROOT/tools/prof_summary.py" "$STATS" 40 > "$OUT/kernels.txt" && head -30 "$OUT/kernels.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/fwd" -o run -- python3 "$ROOT/tools/prof_backbone.py" 1024 3 > "$OUT/fwd.log" 2>&1 || { echo "fwd trace failed"; tail "$OUT/fwd.log"; exit 1; }
python3 "$ROOT/tools/fwd_breakdown.py" $(find "$OUT/fwd" -name '*kernel_trace.csv' | head -1) > "$OUT/forward_breakdown.txt" && cat "$OUT/forward_breakdown.txt"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-extra > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-extra > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; exit 1; }
python3 "$ROOT/tools/pmc_traffic.py" $(find "$OUT/pmc_fetch" -name '*counter_collection.csv' | head -1) \
    $(find "$OUT/pmc_write" -name '*counter_collection.csv' | head -1) "$OUT/traffic.json" > /dev/null && cat "$OUT/traffic.json"
echo "r03_profile $R done"
