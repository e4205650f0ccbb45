#!/bin/bash
# round 6: run a detector test selection against several builds of libmvpose.so (MVPOSE_LIB);
# stops at the first run that does not end as pass (0) or plain test failure (1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/${R06:-r06ab}
SEL="$1"; shift
for lib in "$@"; do
  tag=$(basename $lib .so)
  MVPOSE_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_rtmdet_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "$SEL" > gpurun_out/${R06:-r06ab}/$tag.log 2>&1
  rc=$?
  echo "[$tag] rc=$rc $(tail -1 gpurun_out/${R06:-r06ab}/$tag.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
