#!/bin/bash
# Leg A/B over builds of libwiser_hip.so (WISER_HIP_LIB; "" = the tree's own):
# scripts/leg_run.py per leg and build, twice, the builds interleaved.  Every
# GPU step has its own limit; the first failure ends the script.
# Usage: TAG "LEG..." LIB...
set -eu -o pipefail
TAG=$1; LEGS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for rep in a b; do
  for leg in $LEGS; do
    for lib in "$@"; do
      n=$(basename "${lib:-tree}" .so)
      WISER_HIP_LIB=$lib timeout -k 10 400 python3 scripts/leg_run.py $leg 6 > "$O/${leg}_${n}_$rep.json" 2> "$O/${leg}_${n}_$rep.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'value', d['value'], 'ms/batch', d['ms_per_batch'], 'p50_alone', d.get('p50_alone_ms'), 'frac', d['roofline']['frac'])" "$O/${leg}_${n}_$rep.json" $leg $n
    done
  done
done
