#!/bin/bash
# streaming 32-channel block: bitwise + reference tests, backbone tests, same-box A/B
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -m pytest tests/test_conv_planes_gpu.py -x -q -s -k "tblock32s or basic_block_vs_reference or batch_positions" -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_planes.log 2>&1 || { tail -40 $OUT/pytest_planes.log; exit 1; }
tail -2 $OUT/pytest_planes.log; grep "tblock32s" $OUT/pytest_planes.log
timeout -k 10 300 python3 -u -m pytest tests/test_backbone_gpu.py -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_backbone.log 2>&1 || { tail -40 $OUT/pytest_backbone.log; exit 1; }
tail -2 $OUT/pytest_backbone.log
bash tools/ab_env.sh MVPOSE_NO_TBLOCK32S 2 || exit 1
