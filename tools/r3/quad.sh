#!/bin/bash
# thread-form encode with one put per staged word: parity tests, then encode A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_encode_groups.py tests/test_gpu_stream_path.py > gpurun_out/quad_tests.txt 2>&1 || { tail -30 gpurun_out/quad_tests.txt; exit 1; }
tail -2 gpurun_out/quad_tests.txt
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2" encode noquad= > gpurun_out/ab_quad.txt 2>&1; cat gpurun_out/ab_quad.txt
