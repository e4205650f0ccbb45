#!/bin/bash
# Closing run of the final tree: full GPU suite, smoke, then the closing profile (r04_final.sh).
set -o pipefail
mkdir -p gpurun_out/${TAG:-r04x}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG:-r04x}/pytest.log 2>&1 || { tail -30 gpurun_out/${TAG:-r04x}/pytest.log; exit 1; }
tail -1 gpurun_out/${TAG:-r04x}/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG:-r04x}/smoke.log 2>&1 || { tail gpurun_out/${TAG:-r04x}/smoke.log; exit 1; }
tail -1 gpurun_out/${TAG:-r04x}/smoke.log
bash tools/r04_final.sh
