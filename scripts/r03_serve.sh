#!/bin/bash
# Serving: the server's GPU tests, then the sweep on the C3 stand-in.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_server.py -x -v -m gpu --timeout 120 --timeout-method thread > "$O/pytest_server.log" 2>&1
tail -1 "$O/pytest_server.log"
timeout -k 10 800 python3 scripts/serve_sweep.py 2 > "$O/serve_sweep.txt" 2> "$O/serve_sweep.err"
cat "$O/serve_sweep.txt"
