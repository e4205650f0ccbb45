#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do for v in "" _prio1 _prio3; do
  timeout -k 10 120 ./tools/s32_stamps$v 1024 > $OUT/s32h$v.log 2>&1 || { cat $OUT/s32h$v.log; exit 1; }
  echo "== $v $(head -1 $OUT/s32h$v.log)"; sed -n 2,4p $OUT/s32h$v.log
done; done
