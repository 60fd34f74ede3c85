#!/bin/bash
# GPU parity tests of one variant build (WISER_HIP_LIB), then the A/B of
# scripts/ab_bench.sh (default against every variant).  Usage: TAG VARIANT
set -eu -o pipefail
TAG=$1
V=$2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
WISER_HIP_LIB=$R/wiser_amd/_lib/var_$V/libwiser_hip.so timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu \
    --timeout 120 --timeout-method thread > "$O/pytest_gpu_$V.log" 2>&1 || { tail -40 "$O/pytest_gpu_$V.log"; exit 1; }
tail -1 "$O/pytest_gpu_$V.log"
bash scripts/ab_bench.sh > "$O/ab.txt" 2>&1 || { cat "$O/ab.txt"; exit 1; }
cat "$O/ab.txt"
