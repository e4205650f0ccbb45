#!/bin/bash
# streaming stem2 (libB) roles: no conv1 work / no conv2 work (timing only), s_setprio(2) on conv1 / conv2 waves
set -o pipefail
bash tools/kernel_ab.sh gpurun_out/r04st10 2 libB.so lib_s2x.so lib_s2y.so lib_s2p1.so lib_s2p2.so || exit 1
grep -H stem2 gpurun_out/r04st10/*.txt
