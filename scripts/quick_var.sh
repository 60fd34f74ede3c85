#!/bin/bash
# GPU parity tests (default build), bench, then per-class times for each variant.
# Usage: scripts/quick_var.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 bench.py --no-cpu > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
bash scripts/diag_variants.sh "$TAG/var"
