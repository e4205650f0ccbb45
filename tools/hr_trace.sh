#!/bin/bash
# kernel-trace stats of 3 HRNet-W32 forwards ($3 crops, default 1,024) with library variant $2
set -o pipefail
O=gpurun_out/${1:-hrtrace}; mkdir -p $O; export TMPDIR=/tmp
MVPOSE_LIB=$PWD/multi-camera_3d_pose_estimation_amd/mvpose/${2:-libmvpose.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/hr_fwd.py ${3:-1024} > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
python3 tools/prof_summary.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 40
