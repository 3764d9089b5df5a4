#!/bin/bash
# Round-3 LDS / VALU / wait counters: decode (north star) and thread-form encode (config 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
bash tools/prof_pmc_lds.sh gpurun_out/pmc3d -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 10 > gpurun_out/pmc3d.log 2>&1 || { tail gpurun_out/pmc3d.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc3d decode > gpurun_out/r03_decode_pmc_lds.txt
bash tools/prof_pmc_lds.sh gpurun_out/pmc3e -- python3 tools/kernel_driver.py --kernel encode --config northstar --iters 10 > gpurun_out/pmc3e.log 2>&1 || { tail gpurun_out/pmc3e.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc3e encode > gpurun_out/r03_encode_pmc_lds.txt
cat gpurun_out/r03_decode_pmc_lds.txt gpurun_out/r03_encode_pmc_lds.txt
