#!/bin/bash
# Round-end checks of a build, part A: the GPU suite, smoke, then the counter
# and kernel profiles of every profiled leg (scripts/gpu_prof_legs.sh).  Every
# GPU step has its own limit; the first failure ends the script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -2 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
bash scripts/gpu_prof_legs.sh "${TAG}p" c3 c2 c4_mixed_1to5 c5_phrase single_high realistic_mix
