#!/bin/bash
# SQ stall counters of the backbone kernels: bash tools/pmc_sq.sh NAME
set -o pipefail
N=${1:-sq}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAVES --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/prof_backbone.py" 1024 1 > "$OUT/p1.log" 2>&1 || { echo "p1 failed"; tail "$OUT/p1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/prof_backbone.py" 1024 1 > "$OUT/p2.log" 2>&1 || { echo "p2 failed"; tail "$OUT/p2.log"; exit 1; }
echo done
