#!/bin/bash
# rocprofv3 kernel stats for decode/encode over every BASELINE config (GPU box):
#   bash tools/prof_configs.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/profcfg}
mkdir -p "$OUT"
for k in decode encode; do
  for cfg in northstar config2 config2print config3 config4 config5; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${k}_$cfg" -o run -- \
      python3 tools/kernel_driver.py --kernel $k --config $cfg --iters 10 > "$OUT/${k}_$cfg.log" 2>&1 || { echo "$k $cfg failed"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, re, sys
out = sys.argv[1]
rows = []
for d in sorted(glob.glob(os.path.join(out, "*_*"))):
    if not os.path.isdir(d):
        continue
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        m = re.search(r"namespace\)::([A-Za-z0-9_]+)", r["Name"])
        if m:
            rows.append((os.path.basename(d), m.group(1), r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"]))
with open(os.path.join(out, "configs_kernel_stats.csv"), "w") as fh:
    fh.write("run,kernel,calls,avg_ns,min_ns,max_ns\n")
    for x in rows:
        fh.write(",".join(str(v) for v in x) + "\n")
print(open(os.path.join(out, "configs_kernel_stats.csv")).read())
PY
