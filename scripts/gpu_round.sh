#!/bin/bash
# One GPU round of this session's checks: the GPU suite (optional), smoke,
# the per-class diagnostic and bench.py in the driver's form with the legs
# named.  Each GPU step has its own limit; the first failure ends the script.
# Usage: TAG [--no-tests] [--diag] [bench args...]
set -eu -o pipefail
TAG=$1; shift
TESTS=1; DIAG=0
if [ "${1:-}" = "--no-tests" ]; then TESTS=0; shift; fi
if [ "${1:-}" = "--diag" ]; then DIAG=1; shift; fi
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
if [ $DIAG = 1 ]; then
  timeout -k 10 600 python3 -u scripts/diag_classes.py > "$O/diag.txt" 2> "$O/diag.err"
  cat "$O/diag.txt"
fi
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 "$@" > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", r["frac"], "lean_ms", r.get("lean_kernel_ms"),
      "iso", r.get("isolated_launch_ms"), "per_step GB/s", r.get("achieved_per_step"), "traffic", r.get("traffic"),
      r.get("traffic_stale"), "checked", d.get("parity_checked_queries"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), (v.get("roofline") or {}).get("frac"),
          v.get("vs_weighted_pure_legs"), "checked", v.get("parity_checked_queries"),
          "p50", v.get("p50_ms"), "cpu", (v.get("cpu_baseline") or {}).get("value"))
PY
