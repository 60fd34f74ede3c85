#!/bin/bash
# A/B on the C3 stand-in (per-class segment times, scripts/diag_types.py --wiki)
# and the C2 main leg: the default build against every variant build.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
run() {
  timeout -k 10 400 python3 scripts/diag_types.py --wiki | grep -E "^(mixed|high-high)" || return 1
  timeout -k 10 300 python3 bench.py --no-cpu --no-extra 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('value', d['value'], 'seg', d['kernel_ms_per_batch']['segment'])"
}
for round in 1 2; do
  echo "== default ($round)"; run
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so run
  done
done > "$O/ab_c3.txt" 2>&1
cat "$O/ab_c3.txt"
