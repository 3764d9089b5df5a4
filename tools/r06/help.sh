#!/bin/bash
# Look-backs with the stuck-predecessor help: the encode and read tests
# (default and forced help), then head vs help timing (packed encode, read):
#   bash tools/r06/help.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
T="tests/test_encode_packed.py tests/test_strings.py"
timeout -k 10 400 python3 -u -m pytest $T -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
MHQ_PK_HELP_POLLS=0 timeout -k 10 400 python3 -u -m pytest $T -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/tests_forced.txt" 2>&1 || { tail -30 "$OUT/tests_forced.txt"; exit 1; }
tail -1 "$OUT/tests_forced.txt"
timeout -k 10 400 python3 -u tools/abmulti.py --kernel packed --configs config2,northstar \
  --libs head=build/r06v/lib_new.so,help=build/r06v/lib_help.so,head2=build/r06v/lib_new.so,help2=build/r06v/lib_help.so \
  --reps 5 > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
timeout -k 10 400 python3 -u tools/ab_read.py --libs head=build/r06v/lib_new.so,help=build/r06v/lib_help.so --cases hdr,shuffled \
  --reps 3 > "$OUT/ab_read.txt" 2>&1 || { tail -20 "$OUT/ab_read.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_read.txt"
