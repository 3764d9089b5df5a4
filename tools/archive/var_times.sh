#!/bin/bash
# Times prebuilt variant libraries without the output check (timing builds
# produce wrong output on purpose):  CONFIGS="northstar" bash tools/var_times.sh default name ...
set -o pipefail
for cfg in ${CONFIGS:-northstar}; do
  for name in "$@"; do
    lib=build/var/lib_$name.so
    [ "$name" = default ] && lib=minhq_amd/libmhq_huff.so
    printf "%-10s %-10s " "$name" "$cfg"
    MHQ_LIB_PATH=$lib timeout -k 10 120 python3 tools/kernel_driver.py --kernel ${KERNEL:-decode} --config $cfg \
      --iters ${ITERS:-30} --no-check 2>&1 | grep -v amdgpu.ids | tr '\n' ' ' || exit 1
    echo
  done
done
