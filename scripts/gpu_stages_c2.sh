#!/bin/bash
# Section / pipeline-stage timers of the lean kernel (the -DWSR_PROFILE build,
# make prof) per query class on C2 only.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export WISER_HIP_LIB=$R/wiser_amd/_lib/prof/libwiser_hip.so
timeout -k 10 300 python3 scripts/diag_types.py > "$O/stages_c2.txt" 2>&1
cat "$O/stages_c2.txt"
