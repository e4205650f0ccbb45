#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03s2skip; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_s2conv_gpu.py tests/test_conv_planes_gpu.py tests/test_backbone_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_bench.sh libA.so libB.so 3 --no-cpu-baseline | tee $OUT/ab.txt
