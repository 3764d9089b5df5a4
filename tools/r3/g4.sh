#!/bin/bash
set -o pipefail
bash tools/r3/ab.sh "northstar config2" decode sopen=-DMHQ_DEC_SOPEN=1 > gpurun_out/r3/ab_sopen.txt 2>&1; rc=$?
cat gpurun_out/r3/ab_sopen.txt; [ $rc = 0 ] || exit $rc
bash tools/variants.sh gpurun_out/tl/v tl=-DMHQ_DIAG_TIMELINE tls="-DMHQ_DIAG_TIMELINE -DMHQ_DEC_SOPEN=1" > gpurun_out/tl/build.log 2>&1 || exit 1
for l in tl tls; do
  echo "== $l"; MHQ_LIB_PATH=gpurun_out/tl/v/lib_$l.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 20 2>&1 | grep -v amdgpu.ids
done
