#!/bin/bash
# streaming stem2 (libN) vs the same without input DMA after the first strip (libW, timing only)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04st3 2 libN.so libW.so || exit 1
grep -H stem2 gpurun_out/r04st3/*.txt
