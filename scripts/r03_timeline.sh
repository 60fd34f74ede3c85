#!/bin/bash
# Kernel timeline of the headline bench's timed loop (short run).
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_tl_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$P/tl" -o tl -- \
    python3 "$R/bench.py" --no-cpu --no-extra --check 0 --steps 600 "$@" > "$O/bench_tl.json" 2> "$O/bench_tl.err"
f=$(find "$P/tl" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/timeline.py" "$f" 80 > "$O/timeline.txt"
cat "$O/timeline.txt"
head -c 400 "$O/bench_tl.json"
