#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
for v in etl etlk1 etlk4; do
  for cfg in config2 config4; do
    echo "== $v $cfg"
    MHQ_LIB_PATH=tools/r3/v/lib_$v.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 10 --no-check 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2" decode sopen || exit 1
for l in tl tls; do
  echo "== $l"; MHQ_LIB_PATH=tools/r3/v/lib_$l.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
done
