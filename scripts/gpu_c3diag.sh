#!/bin/bash
# Per-class kernel times on the C3 stand-in (built on the box first).  Usage: scripts/gpu_c3diag.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 500 python3 scripts/diag_types.py --wiki > "$O/diag_c3.txt" 2>&1
cat "$O/diag_c3.txt"
