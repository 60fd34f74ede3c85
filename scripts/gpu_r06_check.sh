#!/bin/bash
# Round 6 check: the register-heap microbenchmark (and its parity against
# WaveHeap), the whole GPU suite, smoke, the 8-rank gloo rehearsal through
# bench.py's own spawn, and bench.py in the driver's form.  Each GPU step has
# its own limit; the first failure ends the script.
# Usage: TAG [--no-n8] [bench args...]
set -eu -o pipefail
TAG=${1:-r06b}; shift || true
N8=1
if [ "${1:-}" = "--no-n8" ]; then N8=0; shift; fi
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 60 ./wiser_amd/_lib/heap_bench > "$O/heap_bench.txt" 2>&1
cat "$O/heap_bench.txt"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
if [ $N8 = 1 ]; then
  timeout -k 10 900 python3 bench.py --gpus 8 --exchange gloo --workload c2 --docs 200000 --vocab 100000 \
      --queries 40000 --steps 40 --warmup 4 --no-extra --no-cpu --check 128 --index-dir /tmp/wiser_n8 \
      > "$O/n8_gloo.json" 2> "$O/n8_gloo.err"
  tail -c 1200 "$O/n8_gloo.json"; echo
fi
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 "$@" > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "p50_alone", d.get("p50_alone_ms"), "frac", r["frac"],
      "lean_ms", r.get("lean_kernel_ms"), "iso", r.get("isolated_launch_ms"), "traffic", r.get("traffic"),
      "checked", d.get("parity_checked_queries"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), v.get("p50_alone_ms"), (v.get("roofline") or {}).get("frac"),
          v.get("vs_weighted_pure_legs"), "checked", v.get("parity_checked_queries"))
PY
