#!/bin/bash
# kernel-level A/B of the non-temporal variants: N0 base, N1 joins' residual/256-ch nt,
# N3 = N1 + trans1 halo nt, N4 = N3 + joins' 64-ch output nt
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/kernel_ab.sh $OUT 2 libN0.so libN1.so libN3.so libN4.so || exit 1
for f in $OUT/*.txt; do echo "== $f"; grep -E "conv1x1_pair|trans1|tconv_kernel<64, 64, 48|^sum" $f; done
