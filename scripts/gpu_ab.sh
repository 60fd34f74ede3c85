#!/bin/bash
# A/B only (no test suite): the default build against every variant build
# under wiser_amd/_lib/var_*.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
bash scripts/ab_bench.sh > "$O/ab.txt" 2>&1
cat "$O/ab.txt"
