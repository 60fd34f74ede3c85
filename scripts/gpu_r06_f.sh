#!/bin/bash
# Round 6 (f): the whole GPU suite and smoke on the tree's build, then leg
# A/Bs: C3 (tree vs noheavy: the heavy-query first bucket), single_high (tree
# vs nosq: the single-term survivor queue), C5 (tree vs nowin: the position
# window).  Each GPU step has its own limit; the first failure ends the script.
set -eu -o pipefail
TAG=${1:-r06f}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c3" "" wiser_amd/_lib/variants/noheavy.so
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "single_high" "" wiser_amd/_lib/variants/nosq.so
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c5_phrase" "" wiser_amd/_lib/variants/nowin.so
