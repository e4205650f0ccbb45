#!/bin/bash
# same-box A/B: N0 = joins as before, N1 = non-temporal residual loads / 256-ch stores in the joins
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_conv_planes_gpu.py tests/test_backbone_gpu.py -q -p no:cacheprovider --timeout 180 --timeout-method thread -k "pair or join or wide or fusion or oracle" > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
bash tools/ab_bench.sh libN0.so libN1.so 3 --no-cpu-baseline 2>&1 | tee $OUT/ab.txt
