#!/bin/bash
# DVFS probe (timing only): tblock32s (B) and tconv16 (C) with each 32x32x16 MFMA replaced by
# two 16x16x32 MFMAs of the same FLOPs, against the shipped library (A)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04m 2 libA.so libB.so libC.so || exit 1
grep -H "tblock32s\|tconv16" gpurun_out/r04m/*.txt
