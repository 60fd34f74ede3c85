#!/bin/bash
# Round 6 (e): the whole GPU suite and smoke, leg A/Bs of the position window
# (C5: tree vs nowin) and the single-term survivor queue (single_high: tree
# vs nosq), then bench.py with the mixed legs.  Each GPU step has its own
# limit; the first failure ends the script.
set -eu -o pipefail
TAG=${1:-r06e}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c5_phrase" "" wiser_amd/_lib/variants/nowin.so
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "single_high" "" wiser_amd/_lib/variants/nosq.so
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --legs c4_mixed_1to5,c5_phrase,realistic_mix,single_high \
    > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "p50_alone", d.get("p50_alone_ms"), "checked", d.get("parity_checked_queries"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), (v.get("roofline") or {}).get("frac"),
          v.get("vs_weighted_pure_legs"), v.get("interleaved"), "checked", v.get("parity_checked_queries"))
PY
