# Detector tuning A/B on one box: det_bench under environment switches.
set -o pipefail
mkdir -p gpurun_out/detab
for cfg in "" "MVPOSE_DET_GEMM=1 MVPOSE_DET_TILE3=8 MVPOSE_CONV_BM64=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 tools/det_bench.py 64 10 2>&1 | grep batch || exit 1
done
