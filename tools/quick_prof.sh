#!/bin/bash
# Backbone-only kernel profile on the GPU box: bash tools/quick_prof.sh NAME [crops] [reps]
set -o pipefail
N=${1:-qp}; CROPS=${2:-1024}; REPS=${3:-3}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 300 python3 -m pytest "$ROOT/tests/test_backbone_gpu.py" -x -q -p no:cacheprovider > "$OUT/test.log" 2>&1 || { echo "backbone test failed"; tail -20 "$OUT/test.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/tools/prof_backbone.py" "$CROPS" "$REPS" > "$OUT/prof.log" 2>&1 || { echo "prof failed"; exit 1; }
python3 "$ROOT/tools/prof_summary.py" "$OUT/run_kernel_stats.csv" 30
