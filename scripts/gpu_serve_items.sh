#!/bin/bash
# Serving points at several work-item lengths (WSR_SERVER_ITEM_BLOCKS).  Every
# GPU step has its own limit; the first failure ends the script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for IB in 63 32 16 8; do
  WSR_SERVER_ITEM_BLOCKS=$IB SWEEP_POINTS="2,8,640,1000;2,8,768,1000;3,8,640,1000" \
    timeout -k 10 300 python3 scripts/serve_sweep.py 2 > "$O/serve_ib$IB.jsonl" 2> "$O/serve_ib$IB.err"
  echo "item blocks $IB"; cat "$O/serve_ib$IB.jsonl"
done
