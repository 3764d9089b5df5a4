#!/bin/bash
# bench.py headline over 2..6 streams, twice each (no CPU leg, no extras).
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do
  for st in 2 3 4 5 6; do
    v=$(timeout -k 10 180 python3 bench.py --no-cpu --no-extras --streams $st --steps 400 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "streams=$st $v"
  done
done
