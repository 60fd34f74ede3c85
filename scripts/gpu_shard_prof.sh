#!/bin/bash
# Where a doc-range shard step's time goes, rehearsed with one rank (the whole
# sharded path over a one-rank RCCL communicator) against the replica: bench
# lines with host phase timers (WSR_HOST_TIMING), then rocprofv3 kernel traces
# of the pure doc-range form and the replica.  Every GPU step has its own
# limit; the first failure ends the script.  Usage: TAG [bench args...]
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_shprof_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd "$R"
WSR_HOST_TIMING=1 timeout -k 10 400 python3 bench.py --mode shard --heavy-blocks 0 --no-extra --no-cpu \
    --steps 1000 "$@" > "$O/shard_hb0.json" 2> "$O/shard_hb0.err"
grep -h "wsr_shard_step host" "$O/shard_hb0.err" || true
WSR_HOST_TIMING=1 timeout -k 10 400 python3 bench.py --mode shard --no-extra --no-cpu \
    --steps 1000 "$@" > "$O/shard_hybrid.json" 2> "$O/shard_hybrid.err"
grep -h "wsr_shard_step host" "$O/shard_hybrid.err" || true
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/hb0" -o hb0 -- \
    python3 "$R/bench.py" --mode shard --heavy-blocks 0 --no-extra --no-cpu --steps 300 "$@" \
    > "$O/prof_hb0.json" 2> "$O/prof_hb0.err"
find "$P/hb0" -name "*kernel_stats.csv" -exec cp {} "$O/hb0_kernel_stats.csv" \;
find "$P/hb0" -name "*kernel_trace.csv" -exec cp {} "$P/hb0_trace.csv" \;
python3 "$R/scripts/trace_overlap.py" "$P/hb0_trace.csv" lean_kernel segment_kernel plan_query_kernel \
    plan_fill_kernel owner_replay_meta_kernel > "$O/hb0_overlap.json"
python3 "$R/scripts/shard_timeline.py" "$P/hb0_trace.csv" > "$O/hb0_timeline.txt" || true
echo "hb0 trace ok"
# two ranks on this one GPU: the gloo rehearsal of every N > 1 form (hybrid,
# pure doc-range, replicas), host exchange pipelined behind the next step
cd "$R"
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --exchange gloo --steps 400 --warmup 20 --no-cpu "$@" \
    > "$O/n2_gloo.json" 2> "$O/n2_gloo.err"
python3 - "$O/n2_gloo.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n2 gloo value", d["value"], {k: v.get("value") for k, v in (d.get("forms") or {}).items()})
PY
