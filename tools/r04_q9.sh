#!/bin/bash
# tconv16 with the next item's DMA pieces interleaved one per tap (libI) vs shipped (libB)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04t9 2 libB.so libI.so || exit 1
grep -H tconv16 gpurun_out/r04t9/*.txt
