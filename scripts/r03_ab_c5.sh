#!/bin/bash
# A/B of variant builds on the C5 phrase leg (and C4), two rounds.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
bench() {
  timeout -k 10 400 python3 bench.py --no-cpu --steps 200 --check 64 --legs c5_phrase,c4_mixed_1to5 2>/dev/null | python3 -c \
    "import json,sys;d=json.loads(sys.stdin.read());L=d['legs'];c=L['c5_phrase'];print('c5', c['value'], c['ms_per_batch'], 'surv', c['survivors_per_batch'], 'chk', c['parity_checked_queries'], 'c4', L['c4_mixed_1to5']['value'])"
}
{
for round in 1 2; do
  echo "== default ($round)"; bench
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so bench
  done
done
} > "$O/ab_c5.txt" 2>&1
cat "$O/ab_c5.txt"
