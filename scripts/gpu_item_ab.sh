#!/bin/bash
# Headline item size A/B (--item-blocks): the driver's 20-step form twice and
# a 1000-step run per size.  Every GPU step has its own limit; the first
# failure ends the script.  Usage: TAG SIZES...
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for n in "$@"; do
  for form in "20 5 a" "20 5 b" "1000 50 c"; do
    set -- $form
    timeout -k 10 300 python3 bench.py --steps $1 --warmup $2 --no-extra --no-cpu --item-blocks $n \
        > "$O/ib${n}_$3.json" 2> "$O/ib${n}_$3.err"
    python3 - "$O/ib${n}_$3.json" "$n" "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("item_blocks", sys.argv[2], "steps", sys.argv[3], "value", d["value"], "ms/step", d["ms_per_step"],
      "frac", r["frac"], "iso", r["isolated_launch_ms"], "p50_alone", d.get("p50_alone_ms"))
PY
  done
done
