#!/bin/bash
# coop encode with K literal groups: parity for each K, then timing per K vs the per-literal kernel
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "encode or round or strings or multidev or golden" > gpurun_out/r3/gpu_tests_enc.txt 2>&1; rc=$?
tail -25 gpurun_out/r3/gpu_tests_enc.txt; [ $rc = 0 ] || exit $rc
VDIR=tools/r3/v bash tools/r3/ab.sh "config2 northstar config4 config5" encode old k1 k2 k4 win2 > gpurun_out/r3/ab_enc.txt 2>&1; rc=$?
cat gpurun_out/r3/ab_enc.txt; exit $rc
