#!/bin/bash
# Kernel-level same-box A/B of in-tree library builds: rocprofv3 kernel trace of the 1,024-crop
# backbone forward (tools/prof_backbone.py) per build, alternating, and the per-family
# breakdown of each run's last forward (tools/fwd_breakdown.py).
#   bash tools/kernel_ab.sh OUTDIR rounds libA.so libB.so ...
set -o pipefail
OUT=$1; R=$2; shift 2
D=multi-camera_3d_pose_estimation_amd/mvpose
mkdir -p $OUT
for r in $(seq 1 $R); do
  for L in "$@"; do
    T=$OUT/${L%.so}.$r
    MVPOSE_LIB=$D/$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $T -o run -- python3 tools/prof_backbone.py 1024 3 > $T.log 2>&1 || { tail $T.log; exit 1; }
    python3 tools/fwd_breakdown.py $(find $T -name '*kernel_trace.csv' | head -1) > $T.txt || exit 1
    echo "== $L round $r: $(tail -1 $T.txt)"
  done
done
