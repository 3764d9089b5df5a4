#!/bin/bash
# A/B of decode (or other kernel) variant libraries on one box.
#   bash tools/r3/ab.sh "<configs>" "<kernel>" name=flags ...
# builds each variant (plus the in-tree library as "base"), then times every
# config on every library twice, interleaved.
set -o pipefail
CFGS=$1; KERN=$2; shift 2
OUT=gpurun_out/ab; mkdir -p $OUT
# VDIR: variants prebuilt in this container (tools/variants.sh VDIR name=flags ...)
if [ -n "$VDIR" ]; then V=$VDIR; else V=$OUT/v; bash tools/variants.sh $V "$@" > $OUT/build.log 2>&1 || { tail -20 $OUT/build.log; exit 1; }; fi
libs="base"
for v in "$@"; do libs="$libs ${v%%=*}"; done
for rep in 1 2; do
  for cfg in $CFGS; do
    for l in $libs; do
      if [ $l = base ]; then lp=minhq_amd/libmhq_huff.so; else lp=$V/lib_$l.so; fi
      r=$(MHQ_LIB_PATH=$lp timeout -k 10 120 python3 tools/kernel_driver.py --kernel $KERN --config $cfg --iters 30 --no-check 2>/dev/null) || { echo "FAIL $l $cfg"; exit 1; }
      echo "$rep $cfg $l $(echo $r | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_launch"], d.get("hbm_frac"))')"
    done
  done
done
