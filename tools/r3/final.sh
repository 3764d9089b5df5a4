#!/bin/bash
# round-3 final evidence on one box: full GPU suite, smoke, then bench + rocprof stats + PMC traffic
set -o pipefail
T=${1:-r03h}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/$T/gpu_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.txt 2>&1 || { tail gpurun_out/$T/smoke.txt; exit 1; }
tail -1 gpurun_out/$T/smoke.txt
bash tools/round_profile.sh gpurun_out/$T
