#!/bin/bash
# Timing experiments: build decode variants with -D flags and time them (run on the GPU box).
#   bash tools/diag_variants.sh name=-DFLAG ...
set -o pipefail
mkdir -p gpurun_out/var
bash tools/variants.sh gpurun_out/var/v "$@" > gpurun_out/var/build.log 2>&1 || { tail gpurun_out/var/build.log; exit 1; }
for v in "$@"; do
  name=${v%%=*}
  echo "== $name"
  MHQ_LIB_PATH=gpurun_out/var/v/lib_$name.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel ${KERNEL:-decode} --config ${CONFIG:-northstar} --iters 20 --no-check 2>&1 | grep -v amdgpu.ids || exit 1
done
