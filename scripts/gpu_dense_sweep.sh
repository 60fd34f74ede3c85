#!/bin/bash
# Per-class times on C2 and the C3 stand-in for several dense-list thresholds
# (WSR_DENSE_DIV) and general-kernel caps (WSR_GEN_PER_CU).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for cfg in "128 4" "1024 4" "4096 4" "1024 8"; do
  set -- $cfg
  echo "== WSR_DENSE_DIV=$1 WSR_GEN_PER_CU=$2" | tee -a "$O/sweep.txt"
  WSR_DENSE_DIV=$1 WSR_GEN_PER_CU=$2 timeout -k 10 400 python3 scripts/diag_types.py --wiki --only mixed >> "$O/sweep.txt" 2>&1
  WSR_DENSE_DIV=$1 WSR_GEN_PER_CU=$2 timeout -k 10 300 python3 scripts/diag_types.py --only mixed >> "$O/sweep.txt" 2>&1
done
cat "$O/sweep.txt"
