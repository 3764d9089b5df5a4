#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "encode or round or strings or multidev or headers or config or golden or symbols" > gpurun_out/r3/gpu_tests_enc.txt 2>&1; rc=$?
tail -25 gpurun_out/r3/gpu_tests_enc.txt; [ $rc = 0 ] || exit $rc
bash tools/r3/ab.sh "config2 northstar config4 config5" encode old=-DMHQ_ENC_COOP=0 > gpurun_out/r3/ab_enc.txt 2>&1; rc=$?
cat gpurun_out/r3/ab_enc.txt; exit $rc
