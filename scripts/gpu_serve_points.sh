#!/bin/bash
# Serving points (dispatch depth, clients, per-client window) on the C3
# stand-in.  Every GPU step has its own limit; the first failure ends the
# script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
SWEEP_POINTS="2,4,1152,1000;2,5,960,1000;2,6,768,1000;3,6,768,1000;3,5,960,1000;2,7,704,1000;3,7,704,1000;3,4,1152,1000" \
  timeout -k 10 400 python3 scripts/serve_sweep.py 2 > "$O/serve_points.jsonl" 2> "$O/serve_points.err"
cat "$O/serve_points.jsonl"
