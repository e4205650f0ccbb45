#!/bin/bash
# Band-halo detector conv: parity tests, same-box A/B against the im2col GEMM (MVPOSE_DET_BAND=0),
# kernel trace of the 128-frame forward.   gpurun -- bash tools/det_band.sh NAME
set -o pipefail
N=${1:-detband}; OUT=gpurun_out/$N; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rtmdet_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for r in 1 2; do
  for b in 0 1; do
    echo "band=$b $(MVPOSE_DET_BAND=$b timeout -k 10 120 python3 tools/det_bench.py 128 10 2>&1 | grep batch)" || exit 1
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/det_bench.py 128 5 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 tools/prof_summary.py $OUT/prof/run_kernel_stats.csv > $OUT/kernels.txt 2>/dev/null || cp $OUT/prof/run_kernel_stats.csv $OUT/kernels.txt
head -12 $OUT/kernels.txt
