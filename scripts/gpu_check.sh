#!/bin/bash
# One GPU round of checks on the current tree: the GPU test suite, smoke, and
# bench.py in the driver's form (--steps 20 --warmup 5) plus optional extra
# bench arguments.  Every GPU step has its own limit; the first failure ends
# the script.  Usage: TAG [--no-tests] [bench args...]
set -eu -o pipefail
TAG=$1; shift
TESTS=1
if [ "${1:-}" = "--no-tests" ]; then TESTS=0; shift; fi
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ $TESTS = 1 ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread \
      -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
  tail -3 "$O/pytest_gpu.log"
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  cat "$O/smoke.log"
fi
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 "$@" > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", r["frac"], "lean_ms", r.get("lean_kernel_ms"),
      "iso", r.get("isolated_launch_ms"), "per_step GB/s", r.get("achieved_per_step"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), (v.get("roofline") or {}).get("frac"))
PY
