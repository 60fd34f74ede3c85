#!/bin/bash
# GPU parity tests of the default build, then the A/B of scripts/ab_bench.sh
# (default against every wiser_amd/_lib/var_* build).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
bash scripts/ab_bench.sh > "$O/ab.txt" 2>&1 || { cat "$O/ab.txt"; exit 1; }
cat "$O/ab.txt"
timeout -k 10 300 python3 bench.py --no-cpu --no-extra > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
