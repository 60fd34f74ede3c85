#!/bin/bash
# GPU tests of the default build, then the c5_phrase leg of the default build
# against every variant build, twice.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
run() {
  timeout -k 10 300 python3 bench.py --no-cpu --legs c5_phrase 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); v=d['legs']['c5_phrase']; print(v['value'], v['segment_ms_per_batch'], v['parity_checked_queries'])"
}
for round in 1 2; do
  echo "== default ($round)"; run
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so run
  done
done > "$O/phrase_ab.txt" 2>&1
cat "$O/phrase_ab.txt"
