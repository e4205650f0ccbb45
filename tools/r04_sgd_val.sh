#!/bin/bash
# SGD kernel change validation: every SGD GPU test + bench's config-5 line
set -o pipefail
mkdir -p gpurun_out/r04sv
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_sgd_gpu.py tests/test_sgd_joint_gpu.py tests/test_sgd_extrinsic_gpu.py > gpurun_out/r04sv/pytest.log 2>&1 || { tail -30 gpurun_out/r04sv/pytest.log; exit 1; }
tail -3 gpurun_out/r04sv/pytest.log
timeout -k 10 240 python3 tools/sgd_line_ab.py | tail -1
