#!/bin/bash
# Decode A/B over prebuilt library variants: VDIR=build/r06t bash tools/r06/abl.sh OUT name... (tile form)
OUT=${1:?}; shift
mkdir -p "$OUT"
for v in "$@"; do
  MHQ_LIB_PATH=${VDIR:-build/r06t}/lib_$v.so timeout -k 10 300 python3 -u tools/decode_ab.py --configs ${CONFIGS:-northstar,config2,config3} ${ABARGS:-} \
    --forms ${FORMS:-tile} --reps ${REPS:-5} > "$OUT/ab_$v.txt" 2>&1 || { echo "FAILED $v"; tail -5 "$OUT/ab_$v.txt"; exit 1; }
  sed "s/^/$v /" "$OUT/ab_$v.txt" | grep config
done
