#!/bin/bash
# A/B on the C3 stand-in: per-class segment times (scripts/diag_types.py --wiki,
# mixed and high x high) for the default build and every variant build under
# wiser_amd/_lib/var_*, two rounds; then the headline bench (--no-cpu
# --no-extra, 3000 steps) per build.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
diag() {
  timeout -k 10 300 python3 scripts/diag_types.py --wiki | grep -E "^(mixed|high-high)|lean stages|sections"
}
bench() {
  timeout -k 10 300 python3 bench.py --no-cpu --no-extra --steps 3000 --check 64 2>/dev/null | python3 -c \
    "import json,sys;d=json.loads(sys.stdin.read());print('value', d['value'], 'ms_per_step', d['ms_per_step'])"
}
{
for round in 1 2; do
  echo "== default ($round)"; diag
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so diag
  done
done
echo "== bench default"; bench
for d in wiser_amd/_lib/var_*/; do
  case $(basename $d) in var_p*|var_notf8) continue;; esac   # timing diagnostics: wrong results
  echo "== bench $(basename $d)"
  WISER_HIP_LIB=$R/$d/libwiser_hip.so bench
done
} > "$O/ab_c3.txt" 2>&1
cat "$O/ab_c3.txt"
