#!/bin/bash
# encode_len pipelined: parity tests, then layout-call A/B against the one-workgroup-per-group kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_encode_groups.py tests/test_gpu_stream_path.py > gpurun_out/lenpipe_tests.txt 2>&1 || { tail -30 gpurun_out/lenpipe_tests.txt; exit 1; }
tail -2 gpurun_out/lenpipe_tests.txt
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config5" layout nopipe= pf2= pf3= pc3= > gpurun_out/ab_lenpipe.txt 2>&1; cat gpurun_out/ab_lenpipe.txt
