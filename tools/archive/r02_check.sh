#!/bin/bash
# Round-2 GPU check: parity tests (one process, per-test timeout), then the layout call at config 4 size.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/kernel_driver.py --kernel layout --config config4 --n 16777216 --iters 10 2>&1 | tail -2 || exit 1
timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 30 2>&1 | tail -1 || exit 1
