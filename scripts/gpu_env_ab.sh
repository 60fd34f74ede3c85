#!/bin/bash
# Headline A/B over one environment knob read at wsr_open (e.g. WSR_HIT_COST):
# the driver's 20-step form twice and a 1000-step run per value.  Every GPU
# step has its own limit; the first failure ends the script.
# Usage: TAG VAR VALUES...
set -eu -o pipefail
TAG=$1; VAR=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in "$@"; do
  for form in "20 5 a" "20 5 b" "1000 50 c"; do
    set -- $form
    env "$VAR=$v" timeout -k 10 300 python3 bench.py --steps $1 --warmup $2 --no-extra --no-cpu \
        > "$O/${VAR}_${v}_$3.json" 2> "$O/${VAR}_${v}_$3.err"
    python3 - "$O/${VAR}_${v}_$3.json" "$VAR=$v" "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "steps", sys.argv[3], "value", d["value"], "ms/step", d["ms_per_step"],
      "frac", r["frac"], "iso", r["isolated_launch_ms"], "p50_alone", d.get("p50_alone_ms"))
PY
  done
done
