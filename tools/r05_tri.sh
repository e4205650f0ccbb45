#!/bin/bash
# Round 5 triangulation pass: certified-solver parity tests, same-box A/B against the round-4
# kernel (libtri_r04.so), rocprofv3 kernel trace + two PMC passes (each with the kernel trace,
# so the clock = GRBM_GUI_ACTIVE / 8 / duration per dispatch) of the tolerance kernel, 1 M frames.
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${1:-r05a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_triangulate_gpu.py tests/test_sgd_extrinsic_gpu.py::test_triangulate_points_f64_dropin_vs_oracle -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_tri.log 2>&1
rc=$?; tail -5 $OUT/pytest_tri.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/tri_tol_ab.py multi-camera_3d_pose_estimation_amd/mvpose/libtri_r04.so multi-camera_3d_pose_estimation_amd/mvpose/libmvpose.so > $OUT/tri_ab.log 2>&1 || { tail $OUT/tri_ab.log; exit 1; }
cat $OUT/tri_ab.log
cd /tmp || exit 1
export MVPOSE_TRI_ONCE_TOL=1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 5 > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 3 > "$OUT/p1.log" 2>&1 || { echo "p1 failed"; tail "$OUT/p1.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 3 > "$OUT/p2.log" 2>&1 || { echo "p2 failed"; tail "$OUT/p2.log"; exit 1; }
unset MVPOSE_TRI_ONCE_TOL
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p3" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 3 > "$OUT/p3.log" 2>&1 || { echo "p3 failed"; tail "$OUT/p3.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p4" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 3 > "$OUT/p4.log" 2>&1 || { echo "p4 failed"; tail "$OUT/p4.log"; exit 1; }
echo "r05_tri done"
