#!/bin/bash
# End-of-session GPU check: parity suite, smoke, the default bench line, the
# driver's short form, the N = 1 sharded rehearsal (RCCL, one rank) and the
# two-rank launcher rehearsal on one GPU (gloo exchange).  Usage: TAG [steps...]
set -eu -o pipefail
TAG=$1; shift
STEPS=${*:-tests bench driver classes shard1 n2}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; exit 1; }
  tail -1 "$O/pytest_gpu.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
fi
if has bench; then
  timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
  head -c 700 "$O/bench.json"; echo
fi
if has driver; then
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu > "$O/bench_driver_form.json" 2> "$O/bench_driver_form.err"
  head -c 400 "$O/bench_driver_form.json"; echo
fi
if has shard1; then
  timeout -k 10 400 python3 bench.py --mode shard --no-extra --no-cpu --steps 500 > "$O/bench_shard_n1.json" 2> "$O/bench_shard_n1.err"
  head -c 400 "$O/bench_shard_n1.json"; echo
fi
if has n2; then
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --exchange gloo --no-cpu --steps 200 --warmup 10 \
      > "$O/bench_n2_gloo.json" 2> "$O/bench_n2_gloo.err" || { tail -40 "$O/bench_n2_gloo.err"; exit 1; }
  head -c 600 "$O/bench_n2_gloo.json"; echo
fi
if has classes; then
  timeout -k 10 300 python3 scripts/diag_types.py --wiki > "$O/classes_c3.txt" 2>&1
  grep -E "^(mixed|high-high)" "$O/classes_c3.txt"
fi
echo done
