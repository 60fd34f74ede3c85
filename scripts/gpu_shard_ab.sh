#!/bin/bash
# One-rank RCCL rehearsal of the sharded forms under several settings (A/B of
# the exchange stream's priority and the step-group size), with host phase
# timers (SET=queues: the hardware-queue count instead; SET=variants VARIANTS="a b": diagnostic builds).  Every GPU step has its own limit; the first failure ends the
# script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
run() {   # name env-assignments... -- bench args...
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" WSR_HOST_TIMING=1 timeout -k 10 300 python3 bench.py --mode shard --no-extra --no-cpu \
      --steps 1000 "$@" > "$O/$name.json" 2> "$O/$name.err"
  python3 - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value", d["value"], "ms/step", d["ms_per_step"], "host", d.get("host_enqueue_ms_per_step"))
PY
  grep -h "wsr_shard_step host\|wsr_comm exchange stream" "$O/$name.err" || true
}
case "${SET:-default}" in
queues)   # hardware queues per process (HIP's default 4): do barrier packets of
          # cross-stream waits in shared queues serialise the batches?
  for q in 4 8 16; do
    run replica_q$q GPU_MAX_HW_QUEUES=$q -- --mode replica
    run hb0_g4_q$q GPU_MAX_HW_QUEUES=$q -- --heavy-blocks 0 --shard-group 4
    run hyb_g4_q$q GPU_MAX_HW_QUEUES=$q -- --shard-group 4
  done ;;
defer)   # owner replays deferred into later lean kernels (default) or not
  run replica X=1 -- --mode replica
  run hb0_g4 X=1 -- --heavy-blocks 0 --shard-group 4
  run hb0_g4_nodefer WSR_REPLAY_DEFER=0 -- --heavy-blocks 0 --shard-group 4
  run hb0_g8 X=1 -- --heavy-blocks 0 --shard-group 8
  run hyb_g4 X=1 -- --shard-group 4
  run hyb_g4_nodefer WSR_REPLAY_DEFER=0 -- --shard-group 4
  run hyb_g2 X=1 -- --shard-group 2 ;;
variants)   # diagnostic builds (scripts/build_variant.py), parity unchecked
  run replica X=1 -- --mode replica
  run hb0_g4 X=1 -- --heavy-blocks 0 --shard-group 4
  for v in ${VARIANTS:-}; do
    run hb0_g4_$v WISER_HIP_LIB=$R/wiser_amd/_lib/variants/$v.so -- --heavy-blocks 0 --shard-group 4 --check 0
  done ;;
*)
  run replica X=1 -- --mode replica
  run hb0_g4 X=1 -- --heavy-blocks 0 --shard-group 4
  run hb0_g4_noprio WSR_COMM_PRIORITY=0 -- --heavy-blocks 0 --shard-group 4
  run hb0_g8 X=1 -- --heavy-blocks 0 --shard-group 8
  run hb0_g1 X=1 -- --heavy-blocks 0 --shard-group 1
  run hyb_g4 X=1 -- --shard-group 4
  run hyb_g4_noprio WSR_COMM_PRIORITY=0 -- --shard-group 4
  run hyb_g8 X=1 -- --shard-group 8
  ;;
esac
