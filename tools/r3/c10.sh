#!/bin/bash
# decode: last-word OR deferred to the next step (default) vs in the end branch (endor); parity first
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_path.py tests/test_multidev.py tests/test_strings.py tests/test_headers.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3/gpu_tests_c10.txt 2>&1; rc=$?
tail -3 gpurun_out/r3/gpu_tests_c10.txt; [ $rc = 0 ] || exit $rc
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config3 config2print" decode endor
