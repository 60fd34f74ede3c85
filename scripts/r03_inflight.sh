#!/bin/bash
# Headline bench at several step counts and host in-flight limits (main leg only).
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for cfg in "600 0" "3000 0" "3000 4" "3000 8" "3000 12"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --no-cpu --no-extra --check 0 --steps $1 --max-inflight $2 \
      > "$O/b_$1_$2.json" 2> "$O/b_$1_$2.err"
  python3 -c "import json,sys; d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1]); print('steps $1 inflight $2', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
done
