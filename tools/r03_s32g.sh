#!/bin/bash
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -m pytest tests/test_conv_planes_gpu.py -x -q -s -k "tblock32s" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_s32.log 2>&1 || { tail -40 $OUT/pytest_s32.log; exit 1; }
tail -1 $OUT/pytest_s32.log
for v in pf22 pf12 pf42 pf23 pf43; do
  timeout -k 10 120 ./tools/s32_stamps_$v 1024 > $OUT/s32_$v.log 2>&1 || { cat $OUT/s32_$v.log; exit 1; }
  echo "== $v $(head -1 $OUT/s32_$v.log)"; sed -n 2,4p $OUT/s32_$v.log
done
bash tools/ab_env.sh MVPOSE_NO_TBLOCK32S 2 || exit 1
