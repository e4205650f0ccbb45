#!/bin/bash
# Same-box A/B of two in-tree library builds through the bench (alternating runs):
#   bash tools/ab_bench.sh libA.so libB.so [rounds] [extra bench args]
set -o pipefail
A=$1; B=$2; R=${3:-2}; shift 3
D=multi-camera_3d_pose_estimation_amd/mvpose
for r in $(seq 1 "$R"); do
  for L in "$A" "$B"; do
    MVPOSE_LIB=$D/$L timeout -k 10 300 python bench.py --no-extra "$@" > gpurun_out/ab_$L.$r.log 2>&1 || exit 1
    echo "$L $(grep -o '"value": [0-9.]*' gpurun_out/ab_$L.$r.log | head -1) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ab_$L.$r.log | head -1)"
  done
done
