#!/bin/bash
# Round 6 final bench: bench.py in the driver's form with every leg (traffic
# from profiles/r06p), twice.  Each GPU step has its own limit; the first
# failure ends the script.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06z
mkdir -p "$O"
cd "$R"
for i in 1 2; do
  timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 > "$O/bench_$i.json" 2> "$O/bench_$i.err"
  python3 - "$O/bench_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "p50", d.get("p50_ms"), "p50_alone", d.get("p50_alone_ms"),
      "frac", r["frac"], "lean_ms", r.get("lean_kernel_ms"), "traffic", r.get("traffic"), "checked", d.get("parity_checked_queries"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), (v.get("roofline") or {}).get("frac"),
          (v.get("roofline") or {}).get("traffic_over_algo"), v.get("vs_weighted_pure_legs"), "checked", v.get("parity_checked_queries"), "p50", v.get("p50_ms"))
PY
done
