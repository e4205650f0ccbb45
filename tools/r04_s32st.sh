#!/bin/bash
# tblock32s output-store diagnostics: baseline (A), lane-contiguous store addresses (B, wrong
# layout, timing only), no output stores (C, timing only)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04s 2 libA.so libB.so libC.so || exit 1
grep -H tblock32s gpurun_out/r04s/*.txt
