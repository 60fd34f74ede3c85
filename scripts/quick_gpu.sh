#!/bin/bash
# Iteration loop on a GPU box: GPU parity tests, bench (no CPU leg), per-class
# kernel times.  Usage: scripts/quick_gpu.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 bench.py --no-cpu > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
timeout -k 10 300 python3 scripts/diag_types.py > "$O/diag.txt" 2>&1
cat "$O/diag.txt"
