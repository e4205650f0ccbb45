#!/bin/bash
# stem2: tile (libA), streaming (libN), streaming + deeper LDS prefetch (libZ)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04st5 2 libA.so libN.so libZ.so || exit 1
grep -H stem2 gpurun_out/r04st5/*.txt
