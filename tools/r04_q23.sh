#!/bin/bash
# prefetch-depth / priority re-tune after the row-reuse changes: tblock64 PF 3 (A1) / 1 (A2);
# tblock32s PF 5/4 (C1), 3/2 (C2), s_setprio(1) on the conv2 waves (C3); shipped libZ
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04t23 2 libZ.so libA1.so libA2.so libC1.so libC2.so libC3.so || exit 1
grep -H "tblock64_kernel\|tblock32s_kernel" gpurun_out/r04t23/*.txt
