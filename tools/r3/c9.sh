#!/bin/bash
# full GPU suite + encode forms per config (c8), then the thread kernel's LDS alignment A/B
set -o pipefail
bash tools/r3/c8.sh || exit 1
VDIR=tools/r3/v bash tools/r3/ab.sh "config2 northstar" encode ea8
