#!/bin/bash
# stem2 diagnostics (timing only): no input DMA after the first tile (U), no output stores (V)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04st2 2 libA.so libU.so libV.so || exit 1
grep -H stem2 gpurun_out/r04st2/*.txt
