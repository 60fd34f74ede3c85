#!/bin/bash
# Diagnostics: the first timed steps of the headline loop (scripts/enqueue_probe.py),
# default and with 8 hardware queues.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 scripts/enqueue_probe.py --steps 2000 > "$O/enqueue_default.txt" 2>&1
cat "$O/enqueue_default.txt"
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 scripts/enqueue_probe.py --steps 2000 > "$O/enqueue_hwq8.txt" 2>&1
cat "$O/enqueue_hwq8.txt"
