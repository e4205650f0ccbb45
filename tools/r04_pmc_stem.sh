#!/bin/bash
# SQ counters of the backbone kernels (stem2 tile = libA, streaming = libN): 2 passes each
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${TAG:-r04ps}; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for L in ${LIBS:-libA libN}; do
  mkdir -p "$OUT/$L"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    (cd /tmp && MVPOSE_LIB=$ROOT/multi-camera_3d_pose_estimation_amd/mvpose/$L.so timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/$L/p$i" -o run -- python3 "$ROOT/tools/prof_backbone.py" 1024 1 > "$OUT/$L/p$i.log" 2>&1) || { echo "pass $L p$i failed"; tail "$OUT/$L/p$i.log"; exit 1; }
  done
  python3 tools/pmc_table.py $(find "$OUT/$L" -name '*counter_collection.csv') > "$OUT/$L/table.txt" 2>&1
  echo "== $L"; grep -A1 "stem2\|tblock32s\|tconv16_kernel<128, 16, 12, 16, 2, 128, false" "$OUT/$L/table.txt"
done
