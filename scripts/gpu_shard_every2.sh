#!/bin/bash
# The sharded path rehearsed with one rank at the default (N = 1) and the
# N = 4 heavy share, heavy queries grouped by the default cadence, then the
# two-rank launcher rehearsal.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for hb in -1 252; do
  timeout -k 10 300 python3 bench.py --mode shard --no-cpu --no-extra --steps 2000 --heavy-blocks $hb \
      > "$O/shard_hb$hb.json" 2> "$O/shard_hb$hb.err" || { tail -30 "$O/shard_hb$hb.err"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/shard_hb$hb.json').read().strip().splitlines()[-1]); print('hb=$hb', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['parity_checked_queries'], json.dumps(d['exchange']))"
done
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --exchange gloo --no-cpu --steps 200 --warmup 10 \
    > "$O/bench_n2_gloo.json" 2> "$O/bench_n2_gloo.err" || { tail -40 "$O/bench_n2_gloo.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_n2_gloo.json').read().strip().splitlines()[-1]); print('n2 gloo', d['value'], d['ms_per_step'], json.dumps(d['exchange']), d.get('parity_checked_queries'), json.dumps(d.get('control')))"
