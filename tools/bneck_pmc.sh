#!/bin/bash
# PMC pass over the fused layer1 (bneck_kernel): MFMA busy, LDS conflicts, waits.
set -o pipefail
N=${1:-bnpmc}; OUT=gpurun_out/$N; mkdir -p $OUT; export TMPDIR=/tmp
export PYTHONPATH=$PWD/multi-camera_3d_pose_estimation_amd BNECK_AB_ONLY=fused
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 tools/bneck_ab.py > $OUT/p1.log 2>&1 || { echo p1 failed; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 tools/bneck_ab.py > $OUT/p2.log 2>&1 || { echo p2 failed; tail -5 $OUT/p2.log; exit 1; }
python3 tools/pmc_table.py $(find $OUT -name "*counter_collection.csv") | grep -i bneck
