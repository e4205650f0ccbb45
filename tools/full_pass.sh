#!/bin/bash
# Full GPU pass: every GPU test (no -x, so one failure does not hide the rest), then the default
# bench.  gpurun -- bash tools/full_pass.sh NAME
set -o pipefail
N=${1:-full}; OUT=gpurun_out/$N; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
