#!/bin/bash
# r06 per-forward breakdown of the 1,024-crop HRNet-W32 forward: a kernel trace of backbone
# forwards only (tools/hr_fwd.py), paired with the graph's launch plan (MACs per launch).
#   gpurun -- bash tools/fwd_breakdown.sh NAME [CROPS]
set -o pipefail
O=gpurun_out/${1:-fwdbd}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/hr_fwd.py ${2:-1024} $O/plan.npz > $O/untraced.txt 2>&1 || { tail -5 $O/untraced.txt; exit 1; }
cat $O/untraced.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/hr_fwd.py ${2:-1024} > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
python3 tools/fwd_breakdown.py $(find $O/prof -name "*kernel_trace.csv" | head -1) $O/plan.npz $O/breakdown.json > $O/breakdown.txt && cat $O/breakdown.txt
