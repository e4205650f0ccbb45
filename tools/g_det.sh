set -o pipefail
N=${1:-det2}
mkdir -p gpurun_out/$N
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_rtmdet_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$N/pytest.log 2>&1; rc=$?
tail -18 gpurun_out/$N/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/det_bench.py 64 10 > gpurun_out/$N/bench.log 2>&1 && cat gpurun_out/$N/bench.log || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$N/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/det_bench.py 64 3 > $GRAFT_REPO_ROOT/gpurun_out/$N/trace.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $(find $GRAFT_REPO_ROOT/gpurun_out/$N/trace -name '*kernel_stats.csv' | head -1) 20
