#!/bin/bash
# Bitmap-intersection threshold sweep (diagnostics): GPU parity of the path,
# then per-class kernel times and the bench value for several WSR_AND_WPB.
# Usage: scripts/and_sweep.sh TAG "0 16 64 ..."
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for v in $2; do
  WSR_AND_WPB=$v timeout -k 10 300 python3 scripts/diag_types.py > "$O/diag_$v.txt" 2>&1
  echo "== WSR_AND_WPB=$v"; grep -E "^(mixed|high-high)" "$O/diag_$v.txt"
  WSR_AND_WPB=$v timeout -k 10 300 python3 bench.py --no-cpu --no-extra > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('value', d['value'], 'seg', d['kernel_ms_per_batch']['segment'])"
done
