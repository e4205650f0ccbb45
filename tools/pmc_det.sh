#!/bin/bash
# SQ counters of the detector kernels: bash tools/pmc_det.sh NAME
set -o pipefail
N=${1:-detsq}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$N
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAVES --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/det_bench.py" 64 1 > "$OUT/p1.log" 2>&1 || { echo "p1 failed"; tail "$OUT/p1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/det_bench.py" 64 1 > "$OUT/p2.log" 2>&1 || { echo "p2 failed"; tail "$OUT/p2.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        if "det_conv_gemm_kernel<192, 3, 1" not in k and "det_conv_gemm_kernel<128, 3, 1" not in k and "dw5" not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c in sorted(d):
        print("   %-24s %.4g" % (c, d[c]))
PY
