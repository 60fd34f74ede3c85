#!/bin/bash
# GPU parity tests, then the main leg (no CPU / extra legs) and per-class kernel
# times on C2 and on the C3 stand-in.  Usage: scripts/gpu_diag.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python3 bench.py --no-cpu --no-extra > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 python3 scripts/diag_types.py > "$O/diag_c2.txt" 2>&1
cat "$O/diag_c2.txt"
timeout -k 10 400 python3 scripts/diag_types.py --wiki > "$O/diag_c3.txt" 2>&1
cat "$O/diag_c3.txt"
