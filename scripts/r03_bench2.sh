#!/bin/bash
# The default bench line (every leg, CPU baselines), then the driver's form.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
head -c 1200 "$O/bench.json"; echo
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu > "$O/bench_driver_form.json" 2> "$O/bench_driver_form.err"
head -c 600 "$O/bench_driver_form.json"; echo
