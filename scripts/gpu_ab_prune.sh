#!/bin/bash
# Pre-probe pruning: GPU parity suite, then A/B of the default build against
# the variant builds (no pruning, the previous commit).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
bash scripts/ab_bench.sh > "$O/ab.txt" 2>&1
cat "$O/ab.txt"
