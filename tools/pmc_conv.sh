#!/bin/bash
# SQ + traffic counters of single BasicBlock planes: bash tools/pmc_conv.sh NAME
set -o pipefail
N=${1:-pc}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for cfg in ${CFGS:-"64 32 24 1" "32 64 48 1"}; do
  tag=$(echo $cfg | tr ' ' '_')
  i=0; mkdir -p "$OUT/$tag"
  for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/$tag/p$i" -o run -- python3 "$ROOT/tools/conv_one.py" $cfg 1024 3 > "$OUT/$tag/p$i.log" 2>&1 || { echo "pass $tag p$i failed"; tail "$OUT/$tag/p$i.log"; exit 1; }
  done
  python3 "$ROOT/tools/pmc_table.py" $(find "$OUT/$tag" -name '*counter_collection.csv') > "$OUT/$tag/table.txt" 2>&1
  echo "== $cfg"; cat "$OUT/$tag/table.txt"
done
echo done
