#!/bin/bash
# Per-class diagnostics for each built variant under wiser_amd/_lib/var_*/ (and
# the default build).  Usage: scripts/diag_variants.sh TAG [class]
set -eu -o pipefail
TAG=$1; CLS=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
ONLY=()
[ -n "$CLS" ] && ONLY=(--only "$CLS")
timeout -k 10 600 python3 scripts/diag_types.py "${ONLY[@]}" > "$O/default.txt" 2>&1
echo "== default"; cat "$O/default.txt"
for d in wiser_amd/_lib/var_*/; do
  v=$(basename "$d")
  WISER_HIP_LIB=$R/$d/libwiser_hip.so timeout -k 10 300 python3 scripts/diag_types.py "${ONLY[@]}" > "$O/$v.txt" 2>&1
  echo "== $v"; cat "$O/$v.txt"
done
