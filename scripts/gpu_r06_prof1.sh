#!/bin/bash
# Round 6 final profiles, part 1: the GPU suite on the frozen build, then
# rocprofv3 kernel stats + EA-counter bytes of the C3 and C2 legs
# (scripts/gpu_prof_legs.sh).  Each GPU step has its own limit; the first
# failure ends the script.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06p
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
bash scripts/gpu_prof_legs.sh r06p c3 c2
