#!/bin/bash
# Replica and one-rank sharded C2 steps against the number of hardware queues
# HIP gives the process (GPU_MAX_HW_QUEUES; 4 is the box default).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra --steps 3000 \
      > "$O/replica_q$q.json" 2> "$O/replica_q$q.err"
  echo "replica q$q $(python3 -c "import json;d=json.loads(open('$O/replica_q$q.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_enqueue_ms_per_step'])")"
  GPU_MAX_HW_QUEUES=$q WSR_HOST_TIMING=1 timeout -k 10 300 python3 -u bench.py --mode shard --no-cpu --no-extra \
      --steps 1000 > "$O/shard_q$q.json" 2> "$O/shard_q$q.err"
  echo "shard q$q $(python3 -c "import json;d=json.loads(open('$O/shard_q$q.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_enqueue_ms_per_step'])")"
  grep "host us" "$O/shard_q$q.err"
done
