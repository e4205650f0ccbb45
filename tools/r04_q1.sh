#!/bin/bash
# (1) SGD Adam-pass load batching (libF) vs shipped (libA) on bench's config-5 line;
# (2) stem2 conv2 prefetch depth 3 (libT, bit-identical) and + two accumulation chains (libS)
set -o pipefail
bash tools/r04_sgd_ab3.sh libF || exit 1
bash tools/kernel_ab.sh gpurun_out/r04st 2 libA.so libT.so libS.so || exit 1
grep -H stem2 gpurun_out/r04st/*.txt
