#!/bin/bash
# tblock32s all row DMAs on the conv2 waves (libE vs libD); stem2 input DMA on the conv2 waves
# only (lib_s2dA) / conv1 waves only (lib_s2dB)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04t14 2 libD.so libE.so lib_s2dA.so lib_s2dB.so || exit 1
grep -H "tblock32s\|stem2" gpurun_out/r04t14/*.txt
