#!/bin/bash
# tblock32s with row reuse: next strip's row DMAs split conv2 / conv1 waves at 12 (shipped, libR) / 8 / 6 / 4
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04t21 3 libR.so libK8.so || exit 1
grep -H tblock32s gpurun_out/r04t21/*.txt
