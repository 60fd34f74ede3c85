#!/bin/bash
# Headline A/B over builds of libwiser_hip.so (WISER_HIP_LIB; "" = the tree's
# own): per build, the driver's 20-step form twice and one 1000-step run,
# the builds interleaved.  Extra bench arguments after "--".  Every GPU step
# has its own limit; the first failure ends the script.
# Usage: TAG LIB... [-- bench args]
set -eu -o pipefail
TAG=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for form in "20 5 a" "1000 50 c" "20 5 b"; do
  set -- $form "$@"
  S=$1; W=$2; F=$3; shift 3
  for lib in "${LIBS[@]}"; do
    n=$(basename "${lib:-tree}" .so)
    WISER_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps $S --warmup $W --no-extra --no-cpu "$@" \
        > "$O/${n}_$F.json" 2> "$O/${n}_$F.err"
    python3 - "$O/${n}_$F.json" "$n" "$S" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "steps", sys.argv[3], "value", d["value"], "ms/step", d["ms_per_step"],
      "lean_ms", r.get("lean_kernel_ms"), "iso", r["isolated_launch_ms"], "p50_alone", d.get("p50_alone_ms"))
PY
  done
done
