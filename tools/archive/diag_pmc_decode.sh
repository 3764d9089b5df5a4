#!/bin/bash
# PMC passes for the decode kernel on the north-star batch and for the inner-loop microbenchmark (GPU box).
set -o pipefail
export TMPDIR=/tmp
bash tools/prof_pmc_lds.sh gpurun_out/pmcd -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 10 > gpurun_out/pmcd.log 2>&1 || { tail gpurun_out/pmcd.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcd decode
bash tools/prof_pmc_lds.sh gpurun_out/pmcu -- ./tools/ubench/ubench 4000 7 16 > gpurun_out/pmcu.log 2>&1 || { tail gpurun_out/pmcu.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcu "ubenchILi7"
