# Detector tuning A/B on one box: det_bench under environment switches.
set -o pipefail
mkdir -p gpurun_out/detab
for cfg in ${DET_AB_CFGS:-"" "MVPOSE_DET_DW=1"}; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 tools/det_bench.py 64 10 2>&1 | grep batch || exit 1
done
