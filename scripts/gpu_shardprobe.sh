#!/bin/bash
# Replica vs one-rank sharded step on C2, with the host enqueue time per step,
# over a few heavy thresholds.  Usage: TAG [heavy-blocks ...]
set -eu -o pipefail
TAG=$1
shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra --steps 3000 > "$O/replica.json" 2> "$O/replica.err"
cat "$O/replica.json"
for hb in "$@"; do
  timeout -k 10 300 python3 -u bench.py --mode shard --heavy-blocks "$hb" --no-cpu --no-extra --steps 1000 \
      > "$O/shard_hb$hb.json" 2> "$O/shard_hb$hb.err"
  cat "$O/shard_hb$hb.json"
done
