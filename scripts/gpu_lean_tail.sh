#!/bin/bash
# Lean-kernel wave start/end times of C3 headline batches (alone and
# pipelined) from a diagnostic build (build it first, in this container:
#   python3 scripts/build_variant.py leantail kernels.hip ... -- see DESIGN §10).
# Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
WISER_HIP_LIB=$R/wiser_amd/_lib/variants/leantail.so timeout -k 10 400 python3 scripts/lean_tail.py \
    > "$O/lean_tail.json" 2> "$O/lean_tail.err"
python3 - "$O/lean_tail.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("alone", "pipelined"):
    for s in d[k][:4]:
        print(k, s)
PY
