#!/bin/bash
# Packed encode by ticket: its tests, then head vs ticket timing: bash tools/r06/ticket.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
true || timeout -k 10 300 python3 -u -m pytest tests/test_encode_packed.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 400 python3 -u tools/abmulti.py --kernel packed --configs config2,northstar \
  --libs head=build/r06v/lib_new.so,ticket=build/r06v/lib_ticket.so,head2=build/r06v/lib_new.so,ticket2=build/r06v/lib_ticket.so \
  --reps 5 > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
timeout -k 10 400 python3 -u tools/r06/sync_probe.py --steps 20 --reps 10 --streams 2,3,4 > "$OUT/probe.txt" 2>&1 || { tail -20 "$OUT/probe.txt"; exit 1; }
grep streams "$OUT/probe.txt"
