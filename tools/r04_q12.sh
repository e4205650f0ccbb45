#!/bin/bash
# DMA issued by one wave per SIMD: shipped before (libB), tconv16 (libC), + s2conv (libS2),
# + trans1 (libT1), + tconv (libTC); kernel-level A/B of the backbone forward
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04t12 2 libB.so libC.so libS2.so libT1.so libTC.so || exit 1
for L in libB libC libS2 libT1 libTC; do echo "== $L"; for r in 1 2; do grep -h "s2conv\|trans1\|tconv_kernel\|tconv16" gpurun_out/r04t12/$L.$r.txt | awk '{s+=$1} END {print s}'; done; done
