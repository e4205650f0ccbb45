#!/bin/bash
# same-box A/B of graph micro-batch settings (MVPOSE_MICRO_BATCH) through the bench:
#   bash tools/r04_mb.sh rounds "cfgA" "cfgB" ...   ("" = default whole-batch segments)
set -o pipefail
R=$1; shift
mkdir -p gpurun_out/mb
for r in $(seq 1 "$R"); do
  i=0
  for c in "$@"; do
    MVPOSE_MICRO_BATCH="$c" timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline > gpurun_out/mb/mb_$i.$r.log 2>&1 || { tail -5 gpurun_out/mb/mb_$i.$r.log; exit 1; }
    echo "[$c] $(grep -o '"value": [0-9.]*' gpurun_out/mb/mb_$i.$r.log | head -1) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/mb/mb_$i.$r.log | head -1)"
    i=$((i+1))
  done
done
