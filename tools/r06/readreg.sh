#!/bin/bash
# The streamed-then-staged read regression on the new library, then on the
# pre-fix library (last: nothing runs after it): bash tools/r06/readreg.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_strings.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/strings_new.txt" 2>&1 || { tail -30 "$OUT/strings_new.txt"; exit 1; }
tail -1 "$OUT/strings_new.txt"
MHQ_LIB_PATH=build/r06v/lib_head.so timeout -k 10 300 python3 -u -m pytest tests/test_strings.py -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -k "streamed_then_staged" > "$OUT/strings_head.txt" 2>&1
echo "head rc=$?"; grep -E "passed|failed|assert|Error" "$OUT/strings_head.txt" | head -8
