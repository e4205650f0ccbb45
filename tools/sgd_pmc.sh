set -o pipefail
OUT=gpurun_out/sgdpmc; mkdir -p $OUT
bash tools/lib_ab.sh gpurun_out/sgdab4 2 "tools/sgd_time.py" libsgda0.so libsgdb1.so libsgdb2.so libsgdb4.so libsgdb5.so || exit 1
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libsgda0.so timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/sgd_time.py > $OUT/trace.log 2>&1 || { echo trace failed; exit 1; }
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libsgda0.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 tools/sgd_time.py > $OUT/p1.log 2>&1 || { echo p1 failed; exit 1; }
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libsgda0.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 tools/sgd_time.py > $OUT/p2.log 2>&1 || { echo p2 failed; exit 1; }
echo done
