#!/bin/bash
# Same-box A/B of in-tree library variants through one timing script (alternating runs):
#   bash tools/lib_ab.sh OUTDIR ROUNDS "script args" libA.so libB.so ...
# e.g. bash tools/lib_ab.sh gpurun_out/sgdab 2 "tools/sgd_bench.py 200" libsgd0.so libsgd1.so
set -o pipefail
OUT=$1; R=$2; CMD=$3; shift 3
D=multi-camera_3d_pose_estimation_amd/mvpose
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for L in "$@"; do
    MVPOSE_LIB=$D/$L timeout -k 10 300 python -u $CMD > "$OUT/$L.$r.log" 2>&1 || { echo "FAILED $L"; tail -5 "$OUT/$L.$r.log"; exit 1; }
    echo "$L.$r $(tail -1 "$OUT/$L.$r.log")"
  done
done
