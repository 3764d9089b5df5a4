#!/bin/bash
# full GPU suite (encode dispatch band), encode times, decode timeline (north star, config 3), ubench 0/7/9/12
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3/gpu_tests_c3.txt 2>&1; rc=$?
tail -3 gpurun_out/r3/gpu_tests_c3.txt; [ $rc = 0 ] || exit $rc
for cfg in northstar config2 config3 config4 config5; do
  timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 30 --no-check 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("encode", d["config"], d["us_per_launch"], d["hbm_frac"])' || exit 1
done
timeout -k 10 200 ./tools/ubench/ubench_loop 1000 0,7,9,12 > gpurun_out/r3/ubench_loop3.txt 2>&1 || { cat gpurun_out/r3/ubench_loop3.txt; exit 1; }
grep -E "variant [0-9]+ waves" gpurun_out/r3/ubench_loop3.txt
for cfg in northstar config3; do
  echo "== timeline $cfg"
  MHQ_LIB_PATH=tools/r3/v/lib_tl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
done
