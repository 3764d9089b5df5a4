#!/bin/bash
# encode_len timing experiments (GPU box): bash tools/diag_len_variants.sh name=-DFLAG ...
set -o pipefail
mkdir -p gpurun_out/lv
bash tools/variants.sh gpurun_out/lv/v "$@" > gpurun_out/lv/build.log 2>&1 || { tail gpurun_out/lv/build.log; exit 1; }
for v in "$@"; do
  name=${v%%=*}
  echo "== $name"
  MHQ_LIB_PATH=gpurun_out/lv/v/lib_$name.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel encode_len --config config2 --iters 20 2>/dev/null || exit 1
done
MHQ_LIB_PATH=gpurun_out/lv/v/lib_base.so timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/lv/pmc -o pmc --output-format csv -- python3 tools/kernel_driver.py --kernel encode_len --config config2 --iters 5 > gpurun_out/lv/pmc.log 2>&1 && python3 tools/pmc_summary.py gpurun_out/lv encode_len
