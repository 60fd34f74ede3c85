#!/bin/bash
# GPU tests, smoke, the default bench (CPU baseline included), then the sharded path
# rehearsed with one rank (native RCCL step, hybrid split).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 python3 bench.py --mode shard --no-cpu --no-extra --steps 2000 > "$O/bench_shard1.json" 2> "$O/bench_shard1.err" || { tail -30 "$O/bench_shard1.err"; exit 1; }
cat "$O/bench_shard1.json"
