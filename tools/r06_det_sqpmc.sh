#!/bin/bash
# round 6: SQ counters per detector kernel (one pmc pass over the det_breakdown plan)
set -o pipefail
O=gpurun_out/${1:-detsq}; B=${2:-512}; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq -o run -- python3 tools/det_breakdown.py run $B $O/plan.npz > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 - $(find $O/sq -name "*counter_collection.csv" | head -1) <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))[:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:25]:
    wc = v.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{k:60s} wave_cyc {wc:12.3e}  valu {v.get('SQ_ACTIVE_INST_VALU',0)/wc:5.2f}  lds {v.get('SQ_ACTIVE_INST_LDS',0)/wc:5.2f}  waitlds {v.get('SQ_WAIT_INST_LDS',0)/wc:5.2f}  waitany {v.get('SQ_WAIT_ANY',0)/wc:5.2f}  anyinst {v.get('SQ_ACTIVE_INST_ANY',0)/wc:5.2f}  valu_insts {v.get('SQ_INSTS_VALU',0):.3e}")
PY
