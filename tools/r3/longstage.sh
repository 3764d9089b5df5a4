#!/bin/bash
# parse-per-thread 2: string tests; long path: decode with windows staged once / nothing decoded (timing bounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_strings.py tests/test_headers.py > gpurun_out/ls_tests.txt 2>&1 || { tail -30 gpurun_out/ls_tests.txt; exit 1; }
tail -2 gpurun_out/ls_tests.txt
VDIR=tools/r3/v bash tools/r3/ab.sh "config5" decode nostage= nodec= > gpurun_out/ab_longstage.txt 2>&1; cat gpurun_out/ab_longstage.txt
