#!/bin/bash
# Kernel-trace statistics (rocprofv3 --kernel-trace --stats) of bench legs run
# alone (scripts/leg_run.py), plus the batch overlap from the trace.  Every
# GPU step has its own limit; the first failure ends the script.
# Usage: TAG LEG...
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_kstats_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd /tmp
for LEG in "$@"; do
  timeout -k 10 400 python3 "$R/scripts/leg_run.py" "$LEG" 1 > "$O/${LEG}_plain.json" 2> "$O/${LEG}_plain.err"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/$LEG/stats" -o stats -- \
      python3 "$R/scripts/leg_run.py" "$LEG" 8 > "$O/${LEG}_stats.json" 2> "$O/${LEG}_stats.err"
  find "$P/$LEG/stats" -name "*kernel_stats.csv" -exec cp {} "$O/${LEG}_kernel_stats.csv" \;
  find "$P/$LEG/stats" -name "*kernel_trace.csv" -exec cp {} "$P/${LEG}_trace.csv" \;
  python3 "$R/scripts/trace_overlap.py" "$P/${LEG}_trace.csv" > "$O/${LEG}_trace_overlap.json"
  echo "== $LEG"; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('value', d['value'], 'ms/batch', d['ms_per_batch'])" "$O/${LEG}_plain.json"
  cut -d, -f1-8 "$O/${LEG}_kernel_stats.csv" | head -12
done
