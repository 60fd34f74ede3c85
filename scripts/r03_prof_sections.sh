#!/bin/bash
# Per-class segment times with the section timers of the WSR_PROFILE build
# (make prof): item setup / segment / finish (replay) / dequeue shares and the
# lean pipeline's stage cycles per driver block.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 scripts/diag_types.py --wiki > "$O/classes_default.txt" 2>&1
WISER_HIP_LIB=$R/wiser_amd/_lib/prof/libwiser_hip.so timeout -k 10 300 python3 scripts/diag_types.py --wiki > "$O/classes_prof.txt" 2>&1
cat "$O/classes_default.txt" "$O/classes_prof.txt"
