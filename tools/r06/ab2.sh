#!/bin/bash
# Round-6 late A/Bs: decode age-skewed tiles (build/r06w lib_s*) and packed
# sizing unroll (build/r06x lib_u*), each with the parity tests of its most
# changed variant.  bash tools/r06/ab2.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
timeout -k 10 420 python3 -u tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print \
  --libs s0=build/r06w/lib_s0.so,s6=build/r06w/lib_s6.so,s10=build/r06w/lib_s10.so,s14=build/r06w/lib_s14.so \
  --reps 5 --check s6,s10,s14 > "$OUT/ab_skew.txt" 2>&1 || { tail -20 "$OUT/ab_skew.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_skew.txt"
MHQ_LIB_PATH=build/r06w/lib_s14.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_decode_long.py \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_s14.txt" 2>&1 || { tail -30 "$OUT/tests_s14.txt"; exit 1; }
tail -1 "$OUT/tests_s14.txt"
MHQ_LIB_PATH=build/r06x/lib_d1u2.so timeout -k 10 300 python3 -u -m pytest tests/test_encode_packed.py \
  -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_d1u2.txt" 2>&1 || { tail -30 "$OUT/tests_d1u2.txt"; exit 1; }
tail -1 "$OUT/tests_d1u2.txt"
timeout -k 10 420 python3 -u tools/abmulti.py --kernel packed --configs config2,northstar,config3 \
  --libs u0=build/r06x/lib_u0.so,u1=build/r06x/lib_u1.so,u2=build/r06x/lib_u2.so,u4=build/r06x/lib_u4.so,d1=build/r06x/lib_d1.so,d1u2=build/r06x/lib_d1u2.so \
  --reps 5 > "$OUT/ab_size.txt" 2>&1 || { tail -20 "$OUT/ab_size.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_size.txt"
