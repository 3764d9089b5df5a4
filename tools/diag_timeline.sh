#!/bin/bash
# Timeline diagnostic build of the decode kernel (run on the GPU box).
set -o pipefail
mkdir -p gpurun_out/tl
bash tools/variants.sh gpurun_out/tl/v tl=-DMHQ_DIAG_TIMELINE "$@" > gpurun_out/tl/build.log 2>&1 || { tail gpurun_out/tl/build.log; exit 1; }
for cfg in northstar; do
  MHQ_LIB_PATH=gpurun_out/tl/v/lib_tl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 20 || exit 1
done
