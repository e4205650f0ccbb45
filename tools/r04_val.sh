#!/bin/bash
# round-4 validation, part 1: every GPU test (no -x: all failures at once) and smoke()
set -o pipefail
OUT=gpurun_out/r04v; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rs -p no:cacheprovider --timeout 300 --timeout-method thread -s > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc2=$?
tail -2 $OUT/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
