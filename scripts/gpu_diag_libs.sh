#!/bin/bash
# scripts/diag_classes.py over builds of libwiser_hip.so (WISER_HIP_LIB; ""
# = the tree's own), one class list, each build in its own process with its
# own limit; the first failure ends the script.  Usage: TAG "CLASS..." LIB...
set -eu -o pipefail
TAG=$1; CLASSES=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for lib in "$@"; do
  n=$(basename "${lib:-tree}" .so)
  WISER_HIP_LIB=$lib timeout -k 10 400 python3 scripts/diag_classes.py $CLASSES > "$O/diag_$n.txt" 2> "$O/diag_$n.err"
  echo "== $n"; cut -c1-200 "$O/diag_$n.txt"
done
