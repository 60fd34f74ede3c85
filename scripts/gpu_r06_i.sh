#!/bin/bash
# Round 6 (i): the heap cost breakdown, the whole GPU suite and smoke, then
# leg A/Bs: C3 (tree vs nosort: the sorted first pass of the replay) and C5
# (tree vs nobag: the bag's pack record beside its start).  Each GPU step has
# its own limit; the first failure ends the script.
set -eu -o pipefail
TAG=${1:-r06i}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 60 ./wiser_amd/_lib/heap_bench > "$O/heap_parts.txt" 2>&1
grep parts "$O/heap_parts.txt"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c3" "" wiser_amd/_lib/variants/nosort.so
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c5_phrase" "" wiser_amd/_lib/variants/nobag.so
