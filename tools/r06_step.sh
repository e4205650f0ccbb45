#!/bin/bash
# round-6 GPU step: the tests named in $1 (pytest node ids / files), then an optional python snippet file $2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R06:-r06x}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest $1 -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -3
if [ -n "$2" ]; then timeout -k 10 600 python3 -u $2 > $O/extra.log 2>&1 || { tail -30 $O/extra.log; exit 1; }; tail -30 $O/extra.log; fi
