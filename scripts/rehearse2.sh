#!/bin/bash
# N=1 bench and a 2-rank rehearsal of the N>1 path on one GPU (gloo: RCCL
# refuses two ranks on one device).  Usage: scripts/rehearse2.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 bench.py --no-cpu > "$O/bench_n1.json" 2> "$O/bench_n1.err"
cat "$O/bench_n1.json"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 \
    > "$O/bench_n2_gloo.json" 2> "$O/bench_n2_gloo.err"
cat "$O/bench_n2_gloo.json"
