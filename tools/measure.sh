#!/bin/bash
# One GPU measurement pass, from the repo root on the GPU box:
#   gpurun -- bash tools/measure.sh NAME
# 1. GPU parity tests  2. triangulation roofline (100k frames)  3. bench (no CPU
# baseline)  4. rocprofv3 kernel trace + stats of a short bench.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
N=${1:-m}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 600 python3 -u -m pytest "$ROOT/tests" -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 "$ROOT/tools/tri_roofline.py" > "$OUT/tri.log" 2>&1 || { echo "tri failed"; tail "$OUT/tri.log"; exit 1; }
cat "$OUT/tri.log"
timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
python3 "$ROOT/tools/prof_summary.py" "$STATS" 40 > "$OUT/kernels.txt" && cat "$OUT/kernels.txt"
echo "measure $N done"
