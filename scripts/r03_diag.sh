#!/bin/bash
# Per-class segment times (C3 stand-in) of the default build and every variant, twice.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
{
for round in 1 2; do
for d in "" wiser_amd/_lib/var_*/; do
  echo "== ${d:-default} ($round)"
  if [ -n "$d" ]; then export WISER_HIP_LIB=$R/$d/libwiser_hip.so; else unset WISER_HIP_LIB; fi
  timeout -k 10 300 python3 scripts/diag_types.py --wiki --repeat 3 | grep -E "^(mixed|high-high)"
done
done
unset WISER_HIP_LIB
} > "$O/diag.txt" 2>&1
cat "$O/diag.txt"
