#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_rtmdet_gpu.py -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "peaked" > $OUT/pytest_det.log 2>&1
rc=$?; grep -E "frame [0-9]+:|peaked detector|passed|failed" $OUT/pytest_det.log | tail -12; [ $rc -le 1 ] || exit $rc
