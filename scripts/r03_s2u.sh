#!/bin/bash
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
head -c 600 "$O/bench.json"; echo
