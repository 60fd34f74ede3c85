#!/bin/bash
# A/B on one box: per-class times and the main bench value of the default
# build and of every variant build (make variant V=... F=...), twice.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
run() {
  timeout -k 10 300 python3 scripts/diag_types.py | grep -E "^(mixed|high-high)" || return 1
  timeout -k 10 300 python3 bench.py --no-cpu --no-extra 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('value', d['value'], 'seg', d['kernel_ms_per_batch']['segment'])"
}
for round in 1 2; do
  echo "== default ($round)"; run
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so run
  done
done
