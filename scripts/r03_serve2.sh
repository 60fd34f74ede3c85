#!/bin/bash
# Serving sweep around 4-6 k queries in flight on the current build (the index
# built first by bench.py's child process).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 bench.py --no-extra --no-cpu --steps 20 --check 0 > /dev/null 2>&1
SWEEP_POINTS="2,8,512,1000;2,10,448,1000;2,12,384,1000;2,6,768,1000;2,16,256,1000;2,10,512,500;2,8,640,1000;2,8,768,1000;2,10,512,1000" \
  timeout -k 10 400 python3 scripts/serve_sweep.py 3 > "$O/serve_sweep.txt" 2>&1
cat "$O/serve_sweep.txt"
