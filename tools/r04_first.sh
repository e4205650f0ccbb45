#!/bin/bash
# round-4 first GPU pass: the changed parity tests, the default bench, a micro-batch A/B
set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_sgd_gpu.py tests/test_triangulate_gpu.py tests/test_sgd_extrinsic_gpu.py tests/test_backbone_gpu.py tests/test_e2e_parity_gpu.py -m gpu -q -rs -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04a/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r04a/pytest_gpu.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err || { tail -20 gpurun_out/r04a/bench.err; exit 1; }
head -c 1500 gpurun_out/r04a/bench.json; echo
bash tools/r04_mb.sh 2 "" "stem:64" "stem:128" "stem:64,branch0:256"
