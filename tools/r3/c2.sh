#!/bin/bash
# encode dispatch by mean: parity (encode tests), kernel times; loop ubench with 2 chains; decode SOPEN A/B
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "encode or round or strings or multidev or golden or config" > gpurun_out/r3/gpu_tests_c2.txt 2>&1; rc=$?
tail -3 gpurun_out/r3/gpu_tests_c2.txt; [ $rc = 0 ] || exit $rc
for cfg in northstar config2 config3 config4 config5; do
  timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 30 --no-check 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("encode", d["config"], d["us_per_launch"], d["hbm_frac"])' || exit 1
done
timeout -k 10 200 ./tools/ubench/ubench_loop 1000 > gpurun_out/r3/ubench_loop2.txt 2>&1 || { cat gpurun_out/r3/ubench_loop2.txt; exit 1; }
grep -E "variant [0-9]+ waves" gpurun_out/r3/ubench_loop2.txt
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config3" decode sopen
