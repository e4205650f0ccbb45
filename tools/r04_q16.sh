#!/bin/bash
# tconv16 structure probes (timing only): shipped (libF), no DMA after the first items (libTN),
# no output stores (MVPOSE_TCONV16_DIAG=2), both
set -o pipefail
OUT=gpurun_out/r04t16; mkdir -p $OUT
D=multi-camera_3d_pose_estimation_amd/mvpose
run() {  # tag lib env...
  local T=$OUT/$1; shift; local L=$1; shift
  env "$@" MVPOSE_LIB=$D/$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $T -o run -- python3 tools/prof_backbone.py 1024 3 > $T.log 2>&1 || { tail $T.log; exit 1; }
  python3 tools/fwd_breakdown.py $(find $T -name '*kernel_trace.csv' | head -1) > $T.txt || exit 1
  echo "== $T"; grep tconv16 $T.txt
}
for r in 1 2; do
  run base.$r libF.so X=0 || exit 1
  run nodma.$r libTN.so X=0 || exit 1
  run nost.$r libF.so MVPOSE_TCONV16_DIAG=2 || exit 1
  run both.$r libTN.so MVPOSE_TCONV16_DIAG=2 || exit 1
done
