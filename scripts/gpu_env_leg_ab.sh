#!/bin/bash
# Leg A/B over environment settings of the tree's build (each "VAR=value ..."
# string, "" = none): scripts/leg_run.py per leg and setting, twice, the
# settings interleaved.  Every GPU step has its own limit; the first failure
# ends the script.  Usage: TAG "LEG..." ENV...
set -eu -o pipefail
TAG=$1; LEGS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for rep in a b; do
  for leg in $LEGS; do
    i=0
    for envs in "$@"; do
      i=$((i+1))
      env $envs timeout -k 10 400 python3 scripts/leg_run.py $leg 6 > "$O/${leg}_e${i}_$rep.json" 2> "$O/${leg}_e${i}_$rep.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], repr(sys.argv[3]), 'value', d['value'], 'ms/batch', d['ms_per_batch'], 'frac', d['roofline']['frac'])" "$O/${leg}_e${i}_$rep.json" $leg "$envs"
    done
  done
done
