#!/bin/bash
# Kernel timelines of the replica and the one-rank sharded C2 steps: how busy
# the device is inside the timed loop (scripts/trace_overlap.py).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_busy_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd /tmp
for m in replica shard; do
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$P/$m" -o tr -- \
      python3 "$R/bench.py" --mode $m --no-cpu --no-extra --check 0 --steps 1500 > "$O/$m.json" 2> "$O/$m.err"
  f=$(find "$P/$m" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/trace_overlap.py" "$f" lean_kernel segment_kernel owner_replay_meta_kernel \
      rcclGenericKernel plan_query_kernel > "$O/${m}_overlap.json"
  echo "$m"
  python3 -c "import json;d=json.load(open('$O/${m}_overlap.json'));print(json.dumps(d['__device__']));print({k:(round(v['avg_duration_ms'],4),round(v['mean_in_flight'],2)) for k,v in d.items() if k!='__device__'})"
done
