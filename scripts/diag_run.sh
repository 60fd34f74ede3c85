#!/bin/bash
# Diagnostics on a GPU box: per-class kernel times with the normal and the
# section-timer builds.  Usage: scripts/diag_run.sh TAG [extra env assignments via env]
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 scripts/diag_types.py > "$O/diag.txt" 2>&1
cat "$O/diag.txt"
WISER_HIP_LIB=$R/wiser_amd/_lib/prof/libwiser_hip.so timeout -k 10 300 python3 scripts/diag_types.py > "$O/diag_prof.txt" 2>&1
cat "$O/diag_prof.txt"
