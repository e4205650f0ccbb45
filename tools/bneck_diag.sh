#!/bin/bash
# fused layer1 timing with library variants (diagnostic builds of bneck.hip)
set -o pipefail
O=gpurun_out/${1:-bndiag}; mkdir -p $O
export PYTHONPATH=$PWD/multi-camera_3d_pose_estimation_amd
for L in libbn_base.so; do
  MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/$L timeout -k 10 120 python -u tools/bneck_ab.py > $O/$L.txt 2>&1 || { tail -3 $O/$L.txt; exit 1; }
  echo "$L: $(grep fused $O/$L.txt | tail -1)"
done
