#!/bin/bash
# Round-5 shard measurements: one-rank RCCL rehearsal of the sharded forms
# against the replica (1,000 steps each; the hybrid at the default one-rank
# threshold, at the N = 8 heavy share, and every query sharded), then two
# ranks on the one GPU with the gloo host exchange (owner replays deferred).
# Every GPU step has its own limit; the first failure ends the script.
# Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
run() {   # name -- bench args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py --no-extra --no-cpu --steps 1000 --warmup 50 "$@" > "$O/$name.json" 2> "$O/$name.err"
  python3 - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ex = d.get("exchange") or {}
print(sys.argv[2], "value", d["value"], "ms/step", d["ms_per_step"], "host", d.get("host_enqueue_ms_per_step"),
      "share", ex.get("heavy_query_share"), "comm", ex.get("comm"))
PY
}
run replica --mode replica
run hybrid_hb64 --mode shard
run hybrid_hb504 --mode shard --heavy-blocks 504
run docshard --mode shard --heavy-blocks 0
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --exchange gloo --steps 300 --warmup 20 --no-cpu \
    > "$O/n2_gloo.json" 2> "$O/n2_gloo.err"
python3 - "$O/n2_gloo.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print("n2 gloo value", d["value"], d["config"]["parallelism"])
for k, v in d.get("forms", {}).items():
    print("  ", k, v["value"], v["ms_per_step"], v.get("hbm_per_rank"))
PY
