#!/bin/bash
# Instruction mix, wait and memory-pipeline counters of the lean kernel on the
# high x high class (C2, or the C3 stand-in with --wiki; 4,096 queries,
# scripts/diag_types.py), one rocprofv3 pass per counter line of
# scripts/counters_hh.txt.  Usage: TAG [--wiki]
set -eu -o pipefail
TAG=$1
WIKI=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_pmc_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd /tmp
# the index (and its log) first, outside the profiler
timeout -k 10 300 python3 "$R/scripts/diag_types.py" $WIKI --only high-high > "$O/diag_hh.txt" 2>&1
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $counters --output-format csv -d "$P/pass$i" -o pmc -- \
      python3 "$R/scripts/diag_types.py" $WIKI --only high-high > "$O/pass$i.txt" 2> "$O/pass$i.err" \
      && echo "pass $i ok: $counters" || { echo "pass $i failed: $counters"; tail -3 "$O/pass$i.err"; exit 1; }
done < "$R/scripts/counters_hh.txt"
python3 "$R/scripts/pmc_summary.py" "$P" > "$O/pmc_hh.json"
python3 -c "
import json; d=json.load(open('$O/pmc_hh.json'))
for k,v in d.items():
    if 'lean' in k: print(k, json.dumps(v, indent=1))
"
