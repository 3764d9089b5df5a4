#!/bin/bash
# WG decode diagnostics (GPU box): the MHQ_DIAG_WG build's stager timeline and decoder split.
set -o pipefail
for cfg in ${CONFIGS:-northstar}; do
  MHQ_LIB_PATH=build/var/lib_${LIB:-wgd}.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
done
