#!/bin/bash
# PMC passes for one kernel (run on the GPU box).  Usage:
#   bash tools/prof_pmc.sh OUTDIR -- python3 tools/kernel_driver.py --kernel decode ...
# Each pass is its own rocprofv3 run (counters never mixed with other traces).
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift; [ "$1" = "--" ] && shift
mkdir -p "$OUT"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $counters -d "$OUT/p$i" -o pmc --output-format csv -- "$@" \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($counters) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $counters"
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
FETCH_SIZE
WRITE_SIZE
LIST
