set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06a
timeout -k 10 600 python3 -u -m pytest tests/test_triangulate_gpu.py tests/test_e2e_parity_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06a/pytest.log 2>&1 || { tail -40 gpurun_out/r06a/pytest.log; exit 1; }
tail -3 gpurun_out/r06a/pytest.log
bash tools/fwd_breakdown.sh r06a_bd 1024
