#!/bin/bash
# Merge class: parity (GPU tests in the merge modes, full-size C3 stand-in),
# per-class kernel times at several WSR_MERGE_RATIO, and the headline bench
# at step counts / in-flight limits.  Usage: TAG [skip_tests]
set -eu -o pipefail
TAG=$1
SKIP=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
if [ -z "$SKIP" ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_prune.py -x -v -k "merge" \
      --timeout 300 --timeout-method thread > "$O/pytest_merge.log" 2>&1
  tail -2 "$O/pytest_merge.log"
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_scale.py -x -v -k "merge_class or c3_full_size_logged" \
      --timeout 600 --timeout-method thread > "$O/pytest_scale.log" 2>&1
  tail -2 "$O/pytest_scale.log"
fi
for r in 0 4 8 16; do
  WSR_MERGE_RATIO=$r timeout -k 10 300 python3 scripts/diag_types.py --wiki --repeat 3 > "$O/c3_classes_m$r.txt" 2>&1
  echo "ratio $r"; grep -E "^(mixed|high-high|low-high|low-low) " "$O/c3_classes_m$r.txt"
done
for r in 0 8; do
  WSR_MERGE_RATIO=$r timeout -k 10 300 python3 scripts/diag_types.py --repeat 3 > "$O/c2_classes_m$r.txt" 2>&1
  echo "C2 ratio $r"; grep -E "^(mixed|high-high) " "$O/c2_classes_m$r.txt"
done
for cfg in "0 600 0" "0 3000 0" "0 3000 8" "8 600 0" "8 3000 8"; do
  set -- $cfg
  WSR_MERGE_RATIO=$1 timeout -k 10 300 python3 bench.py --no-cpu --no-extra --check 64 --steps $2 --max-inflight $3 \
      > "$O/b_m$1_$2_$3.json" 2> "$O/b_m$1_$2_$3.err"
  python3 -c "import json; d=json.loads(open('$O/b_m$1_$2_$3.json').read().strip().splitlines()[-1]); print('merge $1 steps $2 inflight $3', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['kernel_ms_per_batch'])"
done
