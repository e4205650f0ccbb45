#!/bin/bash
# GPU test pass without -x (all failures at once):  gpurun -- bash tools/gt.sh NAME [pytest args...]
set -o pipefail
N=${1:-gt}; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS=()
for a in "$@"; do
    if [ -e "$ROOT/${a%%::*}" ]; then ARGS+=("$ROOT/$a"); else ARGS+=("$a"); fi
done
[ ${#ARGS[@]} -eq 0 ] && ARGS=("$ROOT/tests")
timeout -k 10 900 python3 -u -m pytest "${ARGS[@]}" -m gpu -q -rs -p no:cacheprovider --timeout 120 \
    --timeout-method thread -s > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest_gpu.log" | tail -30
exit $rc
