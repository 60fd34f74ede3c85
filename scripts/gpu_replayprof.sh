#!/bin/bash
# Per-query replay profile (replay_profile.py) on C2 and the C3 stand-in.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export WISER_HIP_LIB=$R/wiser_amd/_lib/var_replayprof/libwiser_hip.so
timeout -k 10 400 python3 scripts/replay_profile.py > "$O/replay_c2.txt" 2>&1 || { tail -20 "$O/replay_c2.txt"; exit 1; }
cat "$O/replay_c2.txt"
timeout -k 10 500 python3 scripts/replay_profile.py --wiki > "$O/replay_c3.txt" 2>&1 || { tail -20 "$O/replay_c3.txt"; exit 1; }
cat "$O/replay_c3.txt"
