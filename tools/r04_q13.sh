#!/bin/bash
# tblock32s: next strip's row DMAs all on the conv1 waves (libK0) / all on the conv2 waves (libK12) vs the 4 / 8 split (libD)
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04t13 2 libD.so libK0.so libK12.so || exit 1
grep -H tblock32s gpurun_out/r04t13/*.txt
