#!/bin/bash
# Shard GPU tests, then the one-rank sharded rehearsal with host phase times.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_shard_gpu.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
WSR_HOST_TIMING=1 timeout -k 10 300 python3 -u bench.py --mode shard --no-cpu --no-extra --steps 2000 \
    > "$O/shard.json" 2> "$O/shard.err"
python3 -c "import json;d=json.loads(open('$O/shard.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['host_enqueue_ms_per_step'],d['p50_ms'])"
grep "host us" "$O/shard.err"
