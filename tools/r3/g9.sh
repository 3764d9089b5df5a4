#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
VDIR=tools/r3/v bash tools/r3/ab.sh "config2" encode k2 x1 x2 x4 x7 || exit 1
for cfg in config2; do echo "== etl $cfg"; MHQ_LIB_PATH=tools/r3/v/lib_etl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode --config $cfg --iters 10 --no-check 2>&1 | grep -v amdgpu.ids || exit 1; done
