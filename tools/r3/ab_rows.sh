#!/bin/bash
# read_strings row (tools/bench_rows.py) on the in-tree library and prebuilt variants in $VDIR, twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for l in base "$@"; do
    if [ $l = base ]; then lp=minhq_amd/libmhq_huff.so; else lp=$VDIR/lib_$l.so; fi
    r=$(MHQ_LIB_PATH=$lp timeout -k 10 200 python3 tools/bench_rows.py --blocks 200 2>/dev/null) || { echo "FAIL $l"; exit 1; }
    echo "$rep $l $(echo $r | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["read_strings_dev"]; print(d["ms"], d["bare_decode_ms"], d["ratio_to_bare_decode"])')"
  done
done
