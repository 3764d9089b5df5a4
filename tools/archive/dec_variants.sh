#!/bin/bash
# Decode parity tests with the default build, then timings of decode build variants (GPU box):
#   bash tools/dec_variants.sh name=-DFLAG ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== default"
timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 20 2>/dev/null || exit 1
[ $# -gt 0 ] && bash tools/diag_variants.sh "$@" 2>&1
