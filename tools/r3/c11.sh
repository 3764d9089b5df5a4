#!/bin/bash
# decode: parity (incl. exact/short regions), deferred last-word OR A/B, exact-region timing
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_path.py tests/test_multidev.py tests/test_strings.py tests/test_headers.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3/gpu_tests_c11.txt 2>&1; rc=$?
tail -3 gpurun_out/r3/gpu_tests_c11.txt; [ $rc = 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/r3/gpu_tests_c11.txt | head -60; exit $rc; }
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config3 config2print" decode endor || exit 1
for lib in base noopt; do
  if [ $lib = base ]; then lp=minhq_amd/libmhq_huff.so; else lp=tools/r3/v/lib_$lib.so; fi
  r=$(MHQ_LIB_PATH=$lp timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 20 --exact 2>/dev/null) || { echo "FAIL exact $lib"; exit 1; }
  echo "exact northstar $lib $(echo $r | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_launch"], d.get("hbm_frac"))')"
done
