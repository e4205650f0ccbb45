#!/bin/bash
# streaming stem2 without DMA (libW) vs also without conv1 work (libX) / without conv2 work (libY); timing only
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04st4 2 libW.so libX.so libY.so || exit 1
grep -H stem2 gpurun_out/r04st4/*.txt
