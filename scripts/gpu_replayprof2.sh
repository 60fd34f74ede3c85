#!/bin/bash
# Replay profile with the heap left out (stream cost alone).  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export WISER_HIP_LIB=$R/wiser_amd/_lib/var_replayprofnoheap/libwiser_hip.so
timeout -k 10 400 python3 scripts/replay_profile.py > "$O/replay_c2_noheap.txt" 2>&1 || { tail -20 "$O/replay_c2_noheap.txt"; exit 1; }
cat "$O/replay_c2_noheap.txt"
