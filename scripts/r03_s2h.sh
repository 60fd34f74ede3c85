#!/bin/bash
# GPU parity suite on the default build, the per-class diag and the pipelined A/B.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
{
for d in "" wiser_amd/_lib/var_*/; do
  echo "== ${d:-default}"
  if [ -n "$d" ]; then export WISER_HIP_LIB=$R/$d/libwiser_hip.so; else unset WISER_HIP_LIB; fi
  timeout -k 10 300 python3 scripts/diag_types.py --wiki | grep -E "^(mixed|high-high)"
done
unset WISER_HIP_LIB
} > "$O/diag.txt" 2>&1
cat "$O/diag.txt"
bash scripts/r03_ab2.sh "$TAG"
