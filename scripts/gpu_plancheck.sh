#!/bin/bash
# Parity tests, then kernel stats of the main leg (plan kernel times) and the bench line.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_plan_$TAG
mkdir -p "$O" "$P"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_scale.py tests/test_gpu_phrase.py \
    > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/stats" -o stats -- \
    python3 "$R/bench.py" --no-cpu --no-extra --steps 3000 > "$O/bench.json" 2> "$O/bench.err"
find "$P/stats" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
python3 -c "
import csv,json
for r in csv.DictReader(open('$O/kernel_stats.csv')): print('  %-40s %6s calls avg %8.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['p50_alone_ms'])"
