#!/bin/bash
# SQ counters of one BasicBlock plane (2 convs x 3 reps, 1024 crops; default tconv 64-ch 32x24):
#   bash tools/pmc_tconv.sh NAME [C H W kernel-name-filter]
set -o pipefail
N=${1:-pt}; C=${2:-64}; H=${3:-32}; W=${4:-24}; KF=${5:-tconv}; export KF; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/conv_one.py" $C $H $W 0 1024 3 > "$OUT/p$i.log" 2>&1 || { echo "pass p$i failed"; tail "$OUT/p$i.log"; exit 1; }
done
python3 "$ROOT/tools/pmc_table.py" $(find "$OUT" -name '*counter_collection.csv') > "$OUT/table.txt" 2>&1
cat "$OUT/table.txt"
for f in $(find "$OUT" -name '*counter_collection.csv'); do
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if __import__('os').environ['KF'] in r.get('Kernel_Name', '')]
agg = collections.defaultdict(float)
for r in rows:
    agg[r['Counter_Name']] += float(r['Counter_Value'])
n = len({r['Dispatch_Id'] for r in rows}) or 1
print({k: round(v / n, 1) for k, v in agg.items()}, 'dispatches', n)
PY
done
