#!/bin/bash
# Two ranks on ONE GPU through the launcher bench.py uses at N > 1
# (torch.distributed.run), the sharded path with the gloo host exchange
# (RCCL refuses two ranks on one device): orchestration + results, not speed.
# Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --exchange gloo --no-cpu --steps 200 --warmup 10 \
    > "$O/bench_n2_gloo.json" 2> "$O/bench_n2_gloo.err" || { tail -40 "$O/bench_n2_gloo.err"; exit 1; }
cat "$O/bench_n2_gloo.json"
