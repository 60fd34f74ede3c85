#!/bin/bash
# Shard-path GPU tests, the core parity tests, then replica and one-rank shard
# benches (host phase times).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_shard_gpu.py tests/test_gpu_parity.py > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra --steps 3000 > "$O/replica.json" 2> "$O/replica.err"
tail -1 "$O/replica.json"
WSR_HOST_TIMING=1 timeout -k 10 300 python3 -u bench.py --mode shard --no-cpu --no-extra --steps 2000 \
    > "$O/shard.json" 2> "$O/shard.err"
tail -1 "$O/shard.json"
grep "host us" "$O/shard.err"
