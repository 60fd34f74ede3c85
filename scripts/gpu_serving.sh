#!/bin/bash
# The server's GPU tests, then the serving leg alone.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_server.py -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_server.log" 2>&1 || { tail -40 "$O/pytest_server.log"; exit 1; }
tail -1 "$O/pytest_server.log"
timeout -k 10 400 python3 bench.py --no-cpu --legs serving > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['legs']['serving']))"
