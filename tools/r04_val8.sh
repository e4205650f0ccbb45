#!/bin/bash
# end-of-round validation of the final tree: full GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r04v8
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04v8/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04v8/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04v8/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04v8/smoke.log 2>&1 || { tail -20 gpurun_out/r04v8/smoke.log; exit 1; }
tail -1 gpurun_out/r04v8/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/r04v8/bench.json 2> gpurun_out/r04v8/bench.err || { tail -20 gpurun_out/r04v8/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04v8/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['sgd']['ms_per_iter_M'], d['sgd']['roofline']['frac'])"
