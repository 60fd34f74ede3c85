#!/bin/bash
# Replay stream prefetch depth (kStreamDepth): parity tests with the default
# build, then the high x high class and the C2 main leg per variant.  Usage: TAG variants
set -eu -o pipefail
TAG=$1
shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_shard_gpu.py tests/test_gpu_scale.py > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for v in default "$@"; do
  lib=""
  [ "$v" != default ] && lib="$R/wiser_amd/_lib/var_$v/libwiser_hip.so"
  WISER_HIP_LIB=$lib timeout -k 10 300 python3 scripts/diag_types.py --only high-high --repeat 3 > "$O/c2hh_$v.txt" 2>&1
  echo "C2hh $v: $(grep -E '^high-high' "$O/c2hh_$v.txt" | tail -1)"
  WISER_HIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra --steps 3000 > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  echo "bench $v $(python3 -c "import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d['p50_alone_ms'])")"
done
