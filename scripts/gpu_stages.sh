#!/bin/bash
# The new KAT GPU tests, then per-class section / pipeline-stage timers of the
# lean kernel (the -DWSR_PROFILE build, make prof) on C2 and the C3 stand-in.
# Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_kats.py > "$O/pytest_kats.log" 2>&1 || { tail -30 "$O/pytest_kats.log"; exit 1; }
tail -1 "$O/pytest_kats.log"
export WISER_HIP_LIB=$R/wiser_amd/_lib/prof/libwiser_hip.so
timeout -k 10 300 python3 scripts/diag_types.py > "$O/stages_c2.txt" 2>&1
cat "$O/stages_c2.txt"
timeout -k 10 400 python3 scripts/diag_types.py --wiki > "$O/stages_c3.txt" 2>&1
cat "$O/stages_c3.txt"
