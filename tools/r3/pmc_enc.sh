#!/bin/bash
# PMC passes over the encode kernel (config given), one pass per counter set
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
CFG=${1:-config2}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for lib in base old; do
  if [ $lib = base ]; then lp=minhq_amd/libmhq_huff.so; else lp=tools/r3/v/lib_$lib.so; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    MHQ_LIB_PATH=$lp timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc/$lib$i -o out -- python3 tools/kernel_driver.py --kernel encode --config $CFG --iters 5 --no-check > gpurun_out/pmc/$lib$i.log 2>&1 || { echo "pass $lib $i failed"; tail -5 gpurun_out/pmc/$lib$i.log; exit 1; }
  done
done
echo done
