#!/bin/bash
# round 6: SGD goldens with each setting, then the bench's config-5 sgd line alternating ($@ = env settings)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R06:-r06sgd}; mkdir -p $O
for cfg in "$@"; do
  env $cfg timeout -k 10 400 python3 -u -m pytest tests/test_sgd_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$(echo $cfg | tr ' =' '__').log 2>&1 || { echo "[$cfg] tests failed"; tail -20 $O/pytest_$(echo $cfg | tr ' =' '__').log; exit 1; }
  echo "[$cfg] $(tail -1 $O/pytest_$(echo $cfg | tr ' =' '__').log)"
done
for r in 1 2; do
  for cfg in "$@"; do
    echo "[$cfg] $(env $cfg timeout -k 10 200 python3 tools/sgd_line.py 2>&1 | tail -3 | tr '\n' ' ')" || exit 1
  done
done
