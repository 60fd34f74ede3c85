#!/bin/bash
# Serving diagnosis: the headline loop at smaller batches (the sizes the
# micro-batcher launches), then serving points at dispatch depths 1-3.  Every
# GPU step has its own limit; the first failure ends the script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for B in 1024 2048; do
  timeout -k 10 300 python3 bench.py --batch $B --no-extra --no-cpu --steps 2000 > "$O/batch$B.json" 2> "$O/batch$B.err"
  python3 - "$O/batch$B.json" $B <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("batch", sys.argv[2], "value", d["value"], "ms/step", d["ms_per_step"], "host", d.get("host_enqueue_ms_per_step"),
      "iso", d["roofline"].get("isolated_launch_ms"))
PY
done
SWEEP_POINTS="1,8,640,1000;2,8,640,1000;3,8,640,1000;1,8,640,200;2,6,768,1000" \
  timeout -k 10 300 python3 scripts/serve_sweep.py 2 > "$O/serve_depth.jsonl" 2> "$O/serve_depth.err"
cat "$O/serve_depth.jsonl"
