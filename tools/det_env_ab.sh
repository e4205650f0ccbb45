#!/bin/bash
# Same-box detector A/B over environment settings (det_bench.py, 128 frames, alternating):
#   bash tools/det_env_ab.sh "" "MVPOSE_DET_1X1=8" ...
set -o pipefail
for r in 1 2; do
  for cfg in "$@"; do
    echo "[$cfg] $(env $cfg timeout -k 10 120 python3 tools/det_bench.py 128 10 2>&1 | grep batch)" || exit 1
  done
done
