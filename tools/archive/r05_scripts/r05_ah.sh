#!/bin/bash
# Round 5 call ah: config 4 encode forms (cooperative K, thread form) timed; the final evidence run's tail on retry.
set -o pipefail
OUT=${1:-gpurun_out/r05ah}
mkdir -p "$OUT"
for f in default thread k1 k2 k4 k8; do
  case $f in default) E="";; thread) E="MHQ_ENC_FORM=thread";; k*) E="MHQ_ENC_K=${f#k}";; esac
  env $E timeout -k 10 300 python3 tools/abmulti.py --kernel encode --configs config4 --reps 3 \
    --libs base=minhq_amd/libmhq_huff.so > "$OUT/enc_$f.txt" 2>&1 || { cat "$OUT/enc_$f.txt"; exit 1; }
  echo "$f: $(grep config4 "$OUT/enc_$f.txt")"
done
