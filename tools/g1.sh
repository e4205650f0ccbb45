set -o pipefail
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_conv_planes_gpu.py -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/g1/test.log 2>&1; rc=$?
tail -30 gpurun_out/g1/test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/conv_bench.py 1024 20 2>&1 | tee gpurun_out/g1/conv_bench.log
