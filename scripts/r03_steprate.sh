#!/bin/bash
# Diagnostics: the headline loop's step rate in scripts/enqueue_probe.py and in
# bench.py, with and without the oracle spot check.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
{
echo "== probe"; timeout -k 10 400 python3 scripts/enqueue_probe.py --steps 2000 --window 500 2>&1 | grep -E "total|steps"
echo "== probe + oracle check 256 + warmup 50"; timeout -k 10 300 python3 scripts/enqueue_probe.py --steps 2000 --window 500 --oracle-check 256 --warmup 50 2>&1 | grep -E "total|steps"
for chk in 0 256; do
  echo "== bench --check $chk"
  timeout -k 10 300 python3 bench.py --no-cpu --no-extra --steps 2000 --check $chk 2>/dev/null | python3 -c \
    "import json,sys;d=json.loads(sys.stdin.read());print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'host', d.get('host_enqueue_ms_per_step'))"
done
echo "== bench driver-style (--steps 20 --warmup 5)"
timeout -k 10 300 python3 bench.py --no-cpu --no-extra --steps 20 --warmup 5 2>/dev/null | python3 -c \
    "import json,sys;d=json.loads(sys.stdin.read());print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'host', d.get('host_enqueue_ms_per_step'))"
} > "$O/steprate.txt" 2>&1
cat "$O/steprate.txt"
