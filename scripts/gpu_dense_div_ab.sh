#!/bin/bash
# The dense threshold (WSR_DENSE_DIV: lists of >= span/div postings get a
# probe structure) on the headline, C4 and C5 legs.  Every GPU step has its
# own limit; the first failure ends the script.  Usage: TAG DIV...
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for DIV in "$@"; do
  WSR_DENSE_DIV=$DIV timeout -k 10 500 python3 bench.py --steps 2000 --no-cpu --legs c4_mixed_1to5,c5_phrase \
      > "$O/div$DIV.json" 2> "$O/div$DIV.err"
  python3 - "$O/div$DIV.json" $DIV <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("div", sys.argv[2], "headline", d["value"], "image GB", round(d["image"]["total_bytes"] / 1e9, 2),
      {k: (v.get("value"), v.get("ms_per_batch"), v.get("segment_ms_per_batch")) for k, v in d["legs"].items()})
PY
done
