#!/bin/bash
# A/B of variant builds on two-term workloads only: the headline (3000 steps)
# and the C2 leg, default build and every wiser_amd/_lib/var_*, two rounds.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
bench() {
  timeout -k 10 400 python3 bench.py --no-cpu --steps 3000 --check 256 --legs c2_synthetic_1m 2>/dev/null | python3 -c \
    "import json,sys;d=json.loads(sys.stdin.read());L=d['legs'];print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'iso_seg', d['kernel_ms_per_batch']['segment'], 'c2', L['c2_synthetic_1m']['value'], 'checked', d['parity_checked_queries'], L['c2_synthetic_1m']['parity_checked_queries'])"
}
{
for round in 1 2; do
  echo "== default ($round)"; bench
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so bench
  done
done
} > "$O/ab3.txt" 2>&1
cat "$O/ab3.txt"
