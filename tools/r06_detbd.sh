#!/bin/bash
# round-6 detector per-op breakdown (tools/det_breakdown.sh) + an env A/B on det_bench 512
set -o pipefail
export TMPDIR=/tmp
bash tools/det_breakdown.sh ${BD:-detbd3} 512 > /dev/null && grep -E "dwpw|dw5" gpurun_out/${BD:-detbd3}/breakdown.txt | head -40 && grep "^sum" gpurun_out/${BD:-detbd3}/breakdown.txt
for r in 1 2; do
  for cfg in "$@"; do
    echo "[$cfg] $(env $cfg timeout -k 10 120 python3 tools/det_bench.py 512 5 2>&1 | grep batch)" || exit 1
  done
done
