#!/bin/bash
# Round 6 (d): the phrase and batch-former GPU tests, the C5 leg A/B of the
# position window (tree vs nowin), then bench.py with the mixed legs.  Each
# GPU step has its own limit; the first failure ends the script.
set -eu -o pipefail
TAG=${1:-r06d}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_phrase.py tests/test_shard_gpu.py -m gpu -x -v \
    --timeout 450 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
MIX_PROBE=0 bash scripts/gpu_r06_ab.sh "$TAG" "c5_phrase" "" wiser_amd/_lib/variants/nowin.so
timeout -k 10 900 python3 bench.py --steps 20 --warmup 5 --legs c4_mixed_1to5,c5_phrase,realistic_mix \
    > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "p50_alone", d.get("p50_alone_ms"), "checked", d.get("parity_checked_queries"))
for k, v in (d.get("legs") or {}).items():
    print(k, v.get("value"), v.get("ms_per_batch"), (v.get("roofline") or {}).get("frac"),
          v.get("vs_weighted_pure_legs"), v.get("interleaved"), "checked", v.get("parity_checked_queries"))
PY
