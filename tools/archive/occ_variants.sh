#!/bin/bash
# Decode occupancy variants (GPU box): build each, check + time it on several configs.
#   bash tools/occ_variants.sh name=-DFLAG... ...
set -o pipefail
# the variant libraries are prebuilt in-tree (here: bash tools/variants.sh build/var name=-D... ...)
for v in base= "$@"; do
  name=${v%%=*}
  lib=build/var/lib_$name.so; [ "$name" = base ] && lib=minhq_amd/libmhq_huff.so
  for cfg in ${CONFIGS:-northstar config2 config2print config5}; do
    echo "== $name $cfg"
    MHQ_LIB_PATH=$lib timeout -k 10 120 python3 tools/kernel_driver.py --kernel ${KERNEL:-decode} --config $cfg --iters 20 ${NOCHECK:+--no-check} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
