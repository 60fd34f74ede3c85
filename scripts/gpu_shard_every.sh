#!/bin/bash
# The sharded path rehearsed with one rank at the N = 8 heavy share
# (--heavy-blocks 504): a sharded step per batch against the grouped default
# (--shard-every 0), then the two-rank launcher rehearsal.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for ev in 1 0; do
  timeout -k 10 300 python3 bench.py --mode shard --no-cpu --no-extra --steps 2000 --heavy-blocks 504 \
      --shard-every $ev > "$O/shard_hb504_every$ev.json" 2> "$O/shard_hb504_every$ev.err" || { tail -30 "$O/shard_hb504_every$ev.err"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/shard_hb504_every$ev.json').read().strip().splitlines()[-1]); print('every=$ev', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], json.dumps(d['exchange']))"
done
timeout -k 10 300 python3 bench.py --mode shard --no-cpu --no-extra --steps 2000 > "$O/shard_default.json" 2> "$O/shard_default.err" || { tail -30 "$O/shard_default.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/shard_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], json.dumps(d['exchange']))"
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --exchange gloo --no-cpu --steps 200 --warmup 10 \
    > "$O/bench_n2_gloo.json" 2> "$O/bench_n2_gloo.err" || { tail -40 "$O/bench_n2_gloo.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_n2_gloo.json').read().strip().splitlines()[-1]); print('n2 gloo', d['value'], d['ms_per_step'], json.dumps(d['exchange']), d.get('parity_checked_queries'))"
