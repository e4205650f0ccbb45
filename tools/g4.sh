set -o pipefail
mkdir -p gpurun_out/g4
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_conv_planes_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/g4/test.log 2>&1 || { tail -30 gpurun_out/g4/test.log; exit 1; }
tail -3 gpurun_out/g4/test.log
for d in 0 1 2; do echo "== diag $d"; MVPOSE_TCONV_DIAG=$d timeout -k 10 300 python3 -u tools/conv_bench.py 1024 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/g4/diag$d.log; done
