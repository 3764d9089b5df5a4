#!/bin/bash
# GPU test suite (one process), then smoke
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3/gpu_tests.txt 2>&1; rc=$?
tail -15 gpurun_out/r3/gpu_tests.txt
exit $rc
