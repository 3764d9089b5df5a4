#!/bin/bash
# Instruction counts (SQ_INSTS_*) of decode-kernel variants (GPU box):
#   bash tools/diag_variant_pmc.sh name=-DFLAG ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/vp
bash tools/variants.sh gpurun_out/vp/v "$@" > gpurun_out/vp/build.log 2>&1 || { tail gpurun_out/vp/build.log; exit 1; }
for v in "$@"; do
  name=${v%%=*}
  MHQ_LIB_PATH=gpurun_out/vp/v/lib_$name.so timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES -d gpurun_out/vp/$name -o pmc --output-format csv -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 5 --no-check > gpurun_out/vp/$name.log 2>&1 || { tail gpurun_out/vp/$name.log; exit 1; }
  echo "== $name"; python3 - gpurun_out/vp/$name <<'PY'
import csv, glob, sys
from collections import defaultdict
v = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "decode_kernel" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("  ".join(f"{k}={sum(x)/len(x)/1e6:.2f}M" for k, x in sorted(v.items())))
PY
done
