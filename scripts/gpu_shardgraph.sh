#!/bin/bash
# One-rank sharded step on C2: host time per phase (WSR_HOST_TIMING), eager
# launches against the hipGraph-captured step (WSR_SHARD_GRAPH).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export WSR_HOST_TIMING=1
timeout -k 10 300 python3 -u bench.py --mode shard --no-cpu --no-extra --steps 1000 \
    > "$O/shard_eager.json" 2> "$O/shard_eager.err"
tail -1 "$O/shard_eager.json"
grep "host us" "$O/shard_eager.err"
WSR_SHARD_GRAPH=1 timeout -k 10 300 python3 -u bench.py --mode shard --no-cpu --no-extra --steps 1000 \
    > "$O/shard_graph.json" 2> "$O/shard_graph.err"
tail -1 "$O/shard_graph.json"
grep "host us" "$O/shard_graph.err"
