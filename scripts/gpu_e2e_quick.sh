#!/bin/bash
# GPU parity tests, then the main leg with the end-to-end leg only.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 400 python3 bench.py --no-cpu --legs end_to_end > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['p50_ms']); print(json.dumps(d['legs']['end_to_end']))"
