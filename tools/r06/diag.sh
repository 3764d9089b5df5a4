#!/bin/bash
# Stream-decode counters (a -DMHQ_DIAG_STREAM build) and the plain A/B.
OUT=${1:?}; shift
mkdir -p "$OUT"
MHQ_LIB_PATH=build/r06v/lib_diag.so timeout -k 10 300 python3 -u tools/decode_ab.py --configs ${CONFIGS:-northstar,config2print} \
  --forms stream --diag --reps 1 > "$OUT/diag.txt" 2>&1 || { tail -20 "$OUT/diag.txt"; exit 1; }
cat "$OUT/diag.txt"
timeout -k 10 300 python3 -u tools/decode_ab.py --configs ${CONFIGS:-northstar,config2print} --forms ${FORMS:-tile,stream} \
  > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
