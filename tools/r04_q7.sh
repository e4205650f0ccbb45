#!/bin/bash
# stem2 4+4 (libQ) vs the same without input DMA after the first strip (libR, timing only)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04st7 2 libQ.so libR.so || exit 1
grep -H stem2 gpurun_out/r04st7/*.txt
