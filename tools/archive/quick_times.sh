#!/bin/bash
# GPU parity tests, then decode/encode/encode_len timings on the headline batches (GPU box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for k in decode encode; do
  for cfg in northstar config2; do
    timeout -k 10 120 python3 tools/kernel_driver.py --kernel $k --config $cfg --iters 20 2>/dev/null || exit 1
  done
done
