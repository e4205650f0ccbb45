#!/bin/bash
# round-4 pass b: fp64 issue probe, SGD scalar-camera A/B, the peaked detector parity test,
# backbone forward breakdown
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
D=multi-camera_3d_pose_estimation_amd/mvpose
export TMPDIR=/tmp
timeout -k 10 120 ./tools/fp64_probe > $OUT/fp64_probe.txt 2>&1 || { cat $OUT/fp64_probe.txt; exit 1; }
cat $OUT/fp64_probe.txt
for r in 1 2; do for L in libA.so libB.so; do
  MVPOSE_LIB=$D/$L timeout -k 10 200 python3 tools/sgd_bench.py > $OUT/sgd_$L.$r.log 2>&1 || { tail $OUT/sgd_$L.$r.log; exit 1; }
  echo "$L $(tail -2 $OUT/sgd_$L.$r.log | grep -o '"M": [0-9]*\|"ms_per_iteration": [0-9.]*' | tr '\n' ' ')"
done; done | tee $OUT/sgd_ab.txt
MVPOSE_LIB=$D/libB.so timeout -k 10 400 python3 -u -m pytest tests/test_sgd_gpu.py -q -p no:cacheprovider --timeout 180 --timeout-method thread > $OUT/pytest_sgd.log 2>&1
rc=$?; tail -1 $OUT/pytest_sgd.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_rtmdet_gpu.py -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "peaked or end_to_end" > $OUT/pytest_det.log 2>&1
rc=$?; grep -E "peaked detector|same prior|passed|failed" $OUT/pytest_det.log | tail -6; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_backbone.py 1024 3 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
python3 tools/fwd_breakdown.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) > $OUT/fwd.txt && tail -42 $OUT/fwd.txt
