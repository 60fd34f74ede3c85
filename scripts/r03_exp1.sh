#!/bin/bash
# C3 per-class kernel times and the hh class through the other paths
# (general kernel: WSR_DENSE_RATIO huge; bitmap AND: WSR_AND_WPB huge).
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 scripts/diag_types.py --wiki --repeat 3 > "$O/c3_classes.txt" 2>&1
cat "$O/c3_classes.txt"
WSR_DENSE_RATIO=1e9 timeout -k 10 300 python3 scripts/diag_types.py --wiki --only high-high --repeat 3 > "$O/c3_hh_general.txt" 2>&1
cat "$O/c3_hh_general.txt"
WSR_AND_WPB=1e9 timeout -k 10 300 python3 scripts/diag_types.py --wiki --only high-high --repeat 3 > "$O/c3_hh_and.txt" 2>&1
cat "$O/c3_hh_and.txt"
timeout -k 10 300 python3 scripts/diag_types.py --repeat 3 > "$O/c2_classes.txt" 2>&1
cat "$O/c2_classes.txt"
WSR_DENSE_RATIO=1e9 timeout -k 10 300 python3 scripts/diag_types.py --only high-high --repeat 3 > "$O/c2_hh_general.txt" 2>&1
cat "$O/c2_hh_general.txt"
