#!/bin/bash
# GPU round: parity tests, then a short bench.  Each GPU step has its own time limit.
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-seconds 5 "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $rc
