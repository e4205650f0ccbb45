#!/bin/bash
# Round measurement recipe — run on the GPU box from the repo root:
#   gpurun -- bash tools/profile_round.sh r01
# 1. GPU parity tests  2. default bench (with the CPU baseline)  3. rocprofv3
# kernel trace + stats of the bench  4./5. separate PMC passes FETCH_SIZE and
# WRITE_SIZE (never combined with other tracing) -> traffic json.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
R=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 900 python3 -u -m pytest "$ROOT/tests" -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 900 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
python3 "$ROOT/tools/prof_summary.py" "$STATS" 40 > "$OUT/kernels.txt" && cat "$OUT/kernels.txt"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-extra > "$OUT/pmc_fetch.log" 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-extra > "$OUT/pmc_write.log" 2>&1 || { echo "pmc write failed"; exit 1; }
python3 "$ROOT/tools/pmc_traffic.py" $(find "$OUT/pmc_fetch" -name '*counter_collection.csv' | head -1) \
    $(find "$OUT/pmc_write" -name '*counter_collection.csv' | head -1) "$OUT/traffic.json" > /dev/null && cat "$OUT/traffic.json"
echo "profile_round $R done"
