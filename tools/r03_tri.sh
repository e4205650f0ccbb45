#!/bin/bash
# triangulation tolerance-kernel pass: parity tests (both f32-iteration variants), roofline A/B,
# kernel trace + PMC of the tolerance kernel (1M frames)
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r03t
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -s -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_tri.log 2>&1 || { tail -40 $OUT/pytest_tri.log; exit 1; }
tail -3 $OUT/pytest_tri.log; grep "bit-identical" $OUT/pytest_tri.log
MVPOSE_TRI_F32=4 timeout -k 10 300 python3 -u -m pytest tests/test_triangulate_gpu.py -x -q -s -k tolerance -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_tri_f32x4.log 2>&1 || { tail -40 $OUT/pytest_tri_f32x4.log; exit 1; }
grep -E "bit-identical|passed|failed" $OUT/pytest_tri_f32x4.log
timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > $OUT/tri_roofline.log 2>&1 || exit 1
MVPOSE_TRI_F32=4 timeout -k 10 300 python3 -u tools/tri_roofline.py 1000000 > $OUT/tri_roofline_f32x4.log 2>&1 || exit 1
grep -h "V=2" $OUT/tri_roofline*.log
cd /tmp || exit 1
export MVPOSE_TRI_ONCE_TOL=1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 5 > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail "$OUT/trace.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 2 > "$OUT/p1.log" 2>&1 || { echo "p1 failed"; tail "$OUT/p1.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/tri_once.py" 1000000 2 > "$OUT/p2.log" 2>&1 || { echo "p2 failed"; tail "$OUT/p2.log"; exit 1; }
echo "r03_tri done"
