#!/bin/bash
# Decode diagnostics (GPU box): timeline build + PMC counters on the north-star batch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MHQ_LIB_PATH=build/var/lib_tl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/prof_pmc_lds.sh gpurun_out/pmcd -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 10 > gpurun_out/pmcd.log 2>&1 || { tail gpurun_out/pmcd.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcd decode
