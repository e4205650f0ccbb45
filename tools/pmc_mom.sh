#!/bin/bash
# SQ counters of the moments kernel: bash tools/pmc_mom.sh NAME
set -o pipefail
N=${1:-pm}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 120 python3 "$ROOT/tools/moments_one.py" 512 5 2>&1 | tee "$OUT/time.log" || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/moments_one.py" 512 1 > "$OUT/p$i.log" 2>&1 || { echo "pass p$i failed"; tail "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
d = defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "moments" in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(d): print(f"{k:28s} {d[k]:.4g}")
wc = d.get("SQ_WAVE_CYCLES", 1)
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
    if k in d: print(f"{k:28s} {d[k] / wc:.3f} of wave cycles")
PY
