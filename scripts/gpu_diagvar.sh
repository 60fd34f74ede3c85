#!/bin/bash
# High x high class time under timing-only diagnostic builds (make variant):
# where the lean kernel's time goes.  Usage: TAG variant...
set -eu -o pipefail
TAG=$1
shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in default "$@"; do
  lib=""
  [ "$v" != default ] && lib="$R/wiser_amd/_lib/var_$v/libwiser_hip.so"
  WISER_HIP_LIB=$lib timeout -k 10 300 python3 scripts/diag_types.py --only high-high --repeat 3 > "$O/c2_$v.txt" 2>&1
  echo "C2 $v: $(grep -E '^high-high' "$O/c2_$v.txt" | tail -1)"
  WISER_HIP_LIB=$lib timeout -k 10 400 python3 scripts/diag_types.py --wiki --only high-high --repeat 3 > "$O/c3_$v.txt" 2>&1
  echo "C3 $v: $(grep -E '^high-high' "$O/c3_$v.txt" | tail -1)"
done
