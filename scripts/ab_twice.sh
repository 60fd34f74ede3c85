#!/bin/bash
# A/B: per-class times of the default build and each variant, twice, same box.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
for round in 1 2; do
  echo "== default ($round)"; timeout -k 10 300 python3 scripts/diag_types.py | grep "seg="
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so timeout -k 10 300 python3 scripts/diag_types.py | grep "seg="
  done
done
