#!/bin/bash
# The C2 main leg under several values of one engine environment knob, twice.
# Usage: TAG VAR "v1 v2 ..."
set -eu -o pipefail
TAG=$1
VAR=$2
VALS=$3
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for round in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python3 bench.py --no-cpu --no-extra 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['kernel_ms_per_batch']['segment'], d['image']['dense_bytes'])"
  done
done > "$O/env_sweep.txt" 2>&1
cat "$O/env_sweep.txt"
