#!/bin/bash
# coop encode in 512-thread workgroups: encode tests, then encode forms per config
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "encode or round or strings or golden or config or multidev" > gpurun_out/r3/gpu_tests_c13.txt 2>&1; rc=$?
tail -3 gpurun_out/r3/gpu_tests_c13.txt; [ $rc = 0 ] || exit $rc
for cfg in northstar config2 config3 config4 config5; do
  for form in auto thread coop; do
    case $form in thread) env="MHQ_ENC_FORM=thread";; auto) env="";; coop) env="MHQ_ENC_FORM=coop";; esac
    r=$(env $env timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 30 --no-check 2>/dev/null) || { echo "FAIL $cfg $form"; exit 1; }
    echo "$cfg $form $(echo $r | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_launch"], d.get("hbm_frac"))')"
  done
done
