set -o pipefail
mkdir -p gpurun_out/g3
export TMPDIR=/tmp
for d in 0 1 2 3; do
  echo "== diag $d" | tee -a gpurun_out/g3/diag.log
  MVPOSE_TCONV_DIAG=$d timeout -k 10 300 python3 -u tools/conv_bench.py 1024 20 2>&1 | grep tconv | tee -a gpurun_out/g3/diag.log
done
