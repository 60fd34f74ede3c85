#!/bin/bash
# Round 6 (g): the heap microbenchmark (the lane-local pop; parity against the
# libstdc++-checked register heap), the whole GPU suite and smoke, a C3 / C2
# leg A/B of the heap (tree vs oldheap: round 5's WaveHeap), then bench.py in
# the driver's form with every leg.  Each GPU step has its own limit; the
# first failure ends the script.
set -eu -o pipefail
TAG=${1:-r06g}
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
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c3" "" wiser_amd/_lib/variants/oldheap.so
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "p50_alone", d.get("p50_alone_ms"), "frac", r["frac"],
      "lean_ms", r.get("lean_kernel_ms"), "iso", r.get("isolated_launch_ms"), "checked", d.get("parity_checked_queries"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), v.get("p50_alone_ms"), (v.get("roofline") or {}).get("frac"),
          v.get("vs_weighted_pure_legs"), v.get("interleaved"), "checked", v.get("parity_checked_queries"))
PY
