#!/bin/bash
# Times prebuilt variant libraries (build/var/lib_<name>.so, built here with
# tools/variants.sh build/var name=-DFLAG ...) on the GPU box:
#   KERNEL=decode CONFIGS="northstar config2" bash tools/prebuilt_variants.sh default name ...
set -o pipefail
for cfg in ${CONFIGS:-northstar}; do
  for name in "$@"; do
    lib=build/var/lib_$name.so
    [ "$name" = default ] && lib=minhq_amd/libmhq_huff.so
    echo "== $name $cfg"
    MHQ_LIB_PATH=$lib timeout -k 10 120 python3 tools/kernel_driver.py --kernel ${KERNEL:-decode} --config $cfg \
      --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
