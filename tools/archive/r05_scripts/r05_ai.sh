#!/bin/bash
# Round 5 call ai: encode forms around the thread form's upper bound (kShortMean 40): cooperative vs thread.
set -o pipefail
OUT=${1:-gpurun_out/r05ai}
mkdir -p "$OUT"
C=${CFGS:-config4,uniform:8:80,uniform:24:72,uniform:8:96,uniform:16:112}
for f in default thread; do
  case $f in default) E="";; thread) E="MHQ_ENC_FORM=thread";; esac
  env $E timeout -k 10 600 python3 tools/abmulti.py --kernel encode --configs $C --reps 3 \
    --libs base=minhq_amd/libmhq_huff.so > "$OUT/enc_$f.txt" 2>&1 || { cat "$OUT/enc_$f.txt"; exit 1; }
  echo "== $f"; grep -v amdgpu.ids "$OUT/enc_$f.txt"
done
