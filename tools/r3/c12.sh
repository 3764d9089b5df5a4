#!/bin/bash
set -o pipefail
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config3 config2print" decode steps3 long1
