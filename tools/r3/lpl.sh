#!/bin/bash
# encode_len with several literals per lane: parity tests, then layout-call A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_strings.py tests/test_gpu_stream_path.py tests/test_abi.py > gpurun_out/lpl_tests.txt 2>&1 || { tail -30 gpurun_out/lpl_tests.txt; exit 1; }
tail -2 gpurun_out/lpl_tests.txt
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config5" layout lpl1= w8= lpl4= > gpurun_out/ab_lpl.txt 2>&1; cat gpurun_out/ab_lpl.txt
