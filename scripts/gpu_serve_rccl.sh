#!/bin/bash
# Serving sweep on the C3 stand-in (scripts/serve_sweep.py) and the hybrid
# one-rank rehearsal under RCCL launch settings.  Every GPU step has its own
# limit; the first failure ends the script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 scripts/serve_sweep.py 2 > "$O/serve_sweep.jsonl" 2> "$O/serve_sweep.err"
cat "$O/serve_sweep.jsonl"
hyb() {
  local name=$1; shift
  env "$@" WSR_HOST_TIMING=1 timeout -k 10 300 python3 bench.py --mode shard --no-extra --no-cpu --steps 1000 \
      > "$O/$name.json" 2> "$O/$name.err"
  python3 - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value", d["value"], "ms/step", d["ms_per_step"], "host", d.get("host_enqueue_ms_per_step"))
PY
  grep -h "wsr_shard_step host" "$O/$name.err" || true
}
hyb hyb_mix0 NCCL_GRAPH_MIXING_SUPPORT=0
hyb hyb_launch_group NCCL_LAUNCH_MODE=GROUP
hyb hyb_launch_parallel NCCL_LAUNCH_MODE=PARALLEL
