#!/bin/bash
# The serving leg of the default build against every variant build, twice.
# Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
run() {
  timeout -k 10 300 python3 bench.py --no-cpu --legs serving 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['legs']['serving']))"
}
for round in 1 2; do
  echo "== default ($round)"; run
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so run
  done
done > "$O/serving_ab.txt" 2>&1
cat "$O/serving_ab.txt"
