#!/bin/bash
# encode forms on config 2 / north star: thread, coop with K = 1, 2, 4, 8, auto; coop timeline (config 2)
set -o pipefail
for cfg in config2 northstar; do
  for form in thread auto coop1 coop2 coop4 coop8; do
    case $form in
      thread) env="MHQ_ENC_FORM=thread";; auto) env="";; coop*) env="MHQ_ENC_K=${form#coop}";;
    esac
    r=$(env $env timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 30 --no-check 2>/dev/null) || { echo "FAIL $cfg $form"; exit 1; }
    echo "$cfg $form $(echo $r | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_launch"], d.get("hbm_frac"))')"
  done
done
echo "== etl config2 (K=2)"
MHQ_ENC_K=2 MHQ_LIB_PATH=tools/r3/v/lib_etl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config config2 --iters 10 --no-check 2>&1 | grep -v amdgpu.ids || exit 1
