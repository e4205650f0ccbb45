set -o pipefail
mkdir -p gpurun_out/g2
export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/mb_sweep.py 1024 '{}' '{"stem":32}' '{"stem":64}' '{"stem":128}' '{"branch0":128}' '{"branch0":256}' '{"branch1":256}' '{"branch2":256}' '{"stem":64,"branch0":256,"branch1":256,"branch2":256}' '{}' 2>&1 | tee gpurun_out/g2/mb.log
