#!/bin/bash
# round-6 detector step: GPU tests, then a same-box A/B of environment settings ($@) on det_bench 512
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/${R06:-r06e}
timeout -k 10 600 python3 -u -m pytest tests/test_rtmdet_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R06:-r06e}/pytest.log 2>&1 || { tail -40 gpurun_out/${R06:-r06e}/pytest.log; exit 1; }
tail -2 gpurun_out/${R06:-r06e}/pytest.log
for r in 1 2 3; do
  for cfg in "$@"; do
    echo "[$cfg] $(env $cfg timeout -k 10 120 python3 tools/det_bench.py 512 5 2>&1 | grep batch)" || exit 1
  done
done
