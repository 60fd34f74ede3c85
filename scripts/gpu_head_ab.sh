#!/bin/bash
# The headline in the driver's form (bench.py --steps 20 --warmup 5, no legs,
# no oracle work) over builds of libwiser_hip.so (WISER_HIP_LIB; "" = the
# tree's own), REPS rounds, the builds interleaved.  Each GPU step has its own
# limit; the first failure ends the script.  Usage: TAG REPS LIB...
set -eu -o pipefail
TAG=$1; REPS=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for rep in $(seq 1 "$REPS"); do
  for lib in "$@"; do
    n=$(basename "${lib:-tree}" .so)
    WISER_HIP_LIB=$lib timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu --check 0 \
        > "$O/head_${n}_$rep.json" 2> "$O/head_${n}_$rep.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'p50_alone', d['p50_alone_ms'], 'iso', d['roofline']['isolated_launch_ms'])" "$O/head_${n}_$rep.json" $n
  done
done
