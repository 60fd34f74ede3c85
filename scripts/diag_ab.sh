#!/bin/bash
# A/B of an engine knob on the per-class diagnostics: scripts/diag_ab.sh TAG VAR VALUE_A VALUE_B
set -eu -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
env "$VAR=$A" timeout -k 10 600 python3 scripts/diag_types.py > "$O/diag_A.txt" 2>&1
echo "== $VAR=$A"; cat "$O/diag_A.txt"
env "$VAR=$B" timeout -k 10 600 python3 scripts/diag_types.py > "$O/diag_B.txt" 2>&1
echo "== $VAR=$B"; cat "$O/diag_B.txt"
