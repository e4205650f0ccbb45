#!/bin/bash
# SGD kernel PMC pass (one trajectory, config 5): VALU instruction counts and busy cycles
set -o pipefail
OUT=gpurun_out/r03sgdpmc; mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $ROOT/$OUT/pmc -o run -- python3 $ROOT/tools/sgd_bench.py 20 > $ROOT/$OUT/pmc.log 2>&1 || { tail $ROOT/$OUT/pmc.log; exit 1; }
F=$(find $ROOT/$OUT/pmc -name '*counter_collection.csv' | head -1)
python3 - "$F" <<'PY'
import csv,sys,collections
agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=r['Kernel_Name']
    if 'sgd_kernel' not in k: continue
    agg[k][r['Counter_Name']]+=float(r['Counter_Value']); n[(k,r['Counter_Name'])]+=1
for k,v in agg.items():
    c=n[(k,'SQ_WAVES')]
    print(k[:60], {kk: round(vv/max(1,c),1) for kk,vv in v.items()})
PY
