#!/bin/bash
# RTMDet-m per-op breakdown: kernel trace + FETCH_SIZE / WRITE_SIZE passes of tools/det_breakdown.py run
set -o pipefail
O=gpurun_out/${1:-detbd}; B=${2:-512}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/det_breakdown.py run $B $O/plan.npz > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/det_breakdown.py run $B $O/plan2.npz > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/det_breakdown.py run $B $O/plan3.npz > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python3 tools/det_breakdown.py report $(find $O/trace -name "*kernel_trace.csv" | head -1) $O/plan.npz $(find $O/fetch -name "*counter_collection.csv" | head -1) $(find $O/write -name "*counter_collection.csv" | head -1) > $O/breakdown.txt && cat $O/breakdown.txt
