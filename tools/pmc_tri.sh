#!/bin/bash
# Triangulation kernel counters: bash tools/pmc_tri.sh NAME  (separate --pmc passes)
set -o pipefail
N=${1:-pt}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -oE "SQ_INSTS_VALU[A-Z0-9_]*F64[A-Z0-9_]*" "$OUT/counters.txt" | sort -u > "$OUT/f64_counters.txt" || true
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/tools/tri_once.py" 100000 5 > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/tri_once.py" 100000 2 > "$OUT/p1.log" 2>&1 || { echo "p1 failed"; tail "$OUT/p1.log"; exit 1; }
F=$(grep -E "ADD_F64|FMA_F64|MUL_F64|TRANS_F64" "$OUT/f64_counters.txt" | head -4 | tr '\n' ' ')
if [ -n "$F" ]; then
  timeout -s KILL 90 rocprofv3 --pmc $F SQ_WAVES --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/tri_once.py" 100000 2 > "$OUT/p2.log" 2>&1 || { echo "p2 failed"; tail "$OUT/p2.log"; exit 1; }
fi
echo "pmc_tri $N done"
