#!/bin/bash
# round-4 status pass: GPU tests (optionally a subset), then the default bench.
#   gpurun -- bash tools/r04_check.sh NAME [pytest targets...]
set -o pipefail
N=${1:-r04}; shift
OUT=gpurun_out/$N
mkdir -p "$OUT"
export TMPDIR=/tmp
T=("$@"); [ ${#T[@]} -eq 0 ] && T=(tests)
timeout -k 10 900 python3 -u -m pytest "${T[@]}" -m gpu -x -q -rs -p no:cacheprovider --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
head -c 3000 "$OUT/bench.json"
