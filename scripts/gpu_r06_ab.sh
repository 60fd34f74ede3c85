#!/bin/bash
# Round 6 A/B: the C3 leg over the deep-pipeline variants (and the tree's
# build), interleaved twice; then the mixed-batch split probe.  Each GPU step
# has its own limit; the first failure ends the script.
# Usage: TAG "LEG..." LIB...
set -eu -o pipefail
TAG=$1; LEGS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
bash scripts/gpu_leg_ab.sh "$TAG" "$LEGS" "$@"
if [ "${MIX_PROBE:-1}" = 1 ]; then
  timeout -k 10 400 python3 scripts/mix_split_probe.py 30 > "$O/mix_split.jsonl" 2> "$O/mix_split.err"
  cat "$O/mix_split.jsonl"
fi
