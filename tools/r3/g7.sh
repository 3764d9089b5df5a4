#!/bin/bash
# coop encode: parity (in-tree lib), then timing vs variants
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "encode or round or strings or multidev or golden" > gpurun_out/r3/gpu_tests_enc.txt 2>&1; rc=$?
tail -5 gpurun_out/r3/gpu_tests_enc.txt; [ $rc = 0 ] || exit $rc
VDIR=tools/r3/v bash tools/r3/ab.sh "config2 northstar config4 config5" encode $VARS > gpurun_out/r3/ab_enc.txt 2>&1; rc=$?
cat gpurun_out/r3/ab_enc.txt; exit $rc
for cfg in config2 config4; do echo "== etl $cfg"; MHQ_LIB_PATH=tools/r3/v/lib_etl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 10 --no-check 2>&1 | grep -v amdgpu.ids || exit 1; done
