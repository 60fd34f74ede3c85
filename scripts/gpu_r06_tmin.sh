#!/bin/bash
# Round 6: the whole GPU suite on the tf-threshold table build (single-term
# and conjunctive lean pipelines), then the C3 and single_high legs against
# the build without the conjunctive table (nolt) and without either (notmin).
# Each GPU step has its own limit; the first failure ends the script.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06t
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
bash scripts/gpu_leg_ab.sh r06t "c3 single_high" "" wiser_amd/_lib/variants/nolt.so wiser_amd/_lib/variants/notmin.so
