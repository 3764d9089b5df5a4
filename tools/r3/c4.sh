#!/bin/bash
# streaming decode: parity (decode tests with MHQ_DEC_STREAM=1), then A/B timings against the tile kernel
set -o pipefail
mkdir -p gpurun_out/r3
MHQ_DEC_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_path.py tests/test_multidev.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/gpu_tests_stream.txt 2>&1; rc=$?
tail -15 gpurun_out/r3/gpu_tests_stream.txt; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
  for cfg in northstar config2 config3 config2print; do
    for st in 0 1; do
      r=$(MHQ_DEC_STREAM=$st timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 30 2>/dev/null) || { echo "FAIL $cfg $st"; exit 1; }
      echo "$rep $cfg stream=$st $(echo $r | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_launch"], d.get("hbm_frac"))')"
    done
  done
done
