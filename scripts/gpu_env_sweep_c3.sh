#!/bin/bash
# The C3 stand-in leg under several values of one engine environment knob.
# Usage: TAG VAR "v1 v2 ..."
set -eu -o pipefail
TAG=$1
VAR=$2
VALS=$3
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 600 python3 bench.py --no-cpu --legs c3_wiki_standin --steps 200 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['legs']['c3_wiki_standin']; print('$VAR=$v', c['value'], c['segment_ms_per_batch'], c['image']['dense_bytes'], c['parity_checked_queries'])"
done > "$O/env_sweep_c3.txt" 2>&1
cat "$O/env_sweep_c3.txt"
