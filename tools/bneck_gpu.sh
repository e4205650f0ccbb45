#!/bin/bash
# GPU check of the fused Bottleneck: its tests, the backbone / join tests, a same-box A/B and a
# kernel-trace profile of the fused layer1.  Usage: bash tools/bneck_gpu.sh NAME
set -o pipefail
N=${1:-bneck}
O=gpurun_out/$N
mkdir -p $O
export PYTHONPATH=$PWD/multi-camera_3d_pose_estimation_amd
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bneck_gpu.py \
  tests/test_conv_planes_gpu.py -k "bneck or layer1 or join or transition or backbone" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/bneck_ab.py > $O/ab.txt 2>&1 && cat $O/ab.txt || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bneck_ab.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print(f\"{float(r['TotalDurationNs'])/1e6:9.2f} ms calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:90]}\")
"
exit $rc
