#!/bin/bash
# A/B of engine env settings on the headline (3000 steps) and the C2 leg, two rounds.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
bench() {
  timeout -k 10 400 env "$@" python3 bench.py --no-cpu --steps 3000 --check 256 --legs c2_synthetic_1m 2>/dev/null | python3 -c \
    "import json,sys;d=json.loads(sys.stdin.read());L=d['legs'];print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'iso_seg', d['kernel_ms_per_batch']['segment'], 'dense_GB', round(d['image']['dense_bytes']/1e9,1), 'c2', L['c2_synthetic_1m']['value'], 'checked', d['parity_checked_queries'], L['c2_synthetic_1m']['parity_checked_queries'])"
}
{
for round in 1 2; do
  for cfg in "X=0" "WSR_DENSE_DIV=4096 WSR_DENSE_BUDGET_GB=64" "WSR_DENSE_DIV=8192 WSR_DENSE_BUDGET_GB=96"; do
    echo "== $cfg ($round)"; bench $cfg
  done
done
} > "$O/envab.txt" 2>&1
cat "$O/envab.txt"
