#!/bin/bash
# One-rank sharded C2 step under runtime variants (comm stream priority,
# hardware queues).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
run() {   # name, env...
  local name=$1
  shift
  env "$@" timeout -k 10 300 python3 -u bench.py --mode shard --no-cpu --no-extra --check 0 --steps 2000 \
      > "$O/$name.json" 2> "$O/$name.err"
  echo "$name $(python3 -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_enqueue_ms_per_step'])")"
}
run base WSR_COMM_PRIORITY=0
run prio WSR_COMM_PRIORITY=1
run q8 GPU_MAX_HW_QUEUES=8
run prio_q8 WSR_COMM_PRIORITY=1 GPU_MAX_HW_QUEUES=8
run base2 WSR_COMM_PRIORITY=0
