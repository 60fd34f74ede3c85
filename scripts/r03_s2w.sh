#!/bin/bash
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
bash scripts/r03_ab3.sh "$TAG"
SWEEP_POINTS="2,8,512,1000;2,10,448,1000;2,12,384,1000;2,6,768,1000;2,16,256,1000;2,10,512,500;2,8,640,1000;2,8,768,1000;2,10,512,1000" \
  timeout -k 10 400 python3 scripts/serve_sweep.py 3 > "$O/serve_sweep.txt" 2>&1
cat "$O/serve_sweep.txt"
