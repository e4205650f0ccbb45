#!/bin/bash
# trans1 rebalance: parity (R1 = the tree) + kernel-level A/B R0 (6 t0 + 2 t1 waves) vs R1 (4 + 4)
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_conv_planes_gpu.py tests/test_backbone_gpu.py -q -p no:cacheprovider --timeout 180 --timeout-method thread -k "transition1 or oracle or fusion" > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/pytest.log | head; exit 1; }
bash tools/kernel_ab.sh $OUT 2 libR0.so libR1.so || exit 1
for f in $OUT/*.txt; do echo "== $f $(grep -E 'trans1' $f) $(tail -1 $f)"; done
