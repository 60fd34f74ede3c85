#!/bin/bash
# Lean-wave segment / item-end times of C3 headline batches from the
# `leanphase` diagnostic build (build it first, in this container:
#   bash scripts/gpu_lean_phase.sh --build).  Usage: TAG | --build
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
if [ "$1" = "--build" ]; then
  python3 scripts/build_variant.py leanphase kernels.hip \
    "  uint32_t n_surv = 0, n_dblk = 0;
  uint32_t shard = wid % kQueueShards, tried = 0;" \
    "  uint32_t n_surv = 0, n_dblk = 0;
  uint64_t t_seg = 0, t_fin = 0, t_fmax = 0, ts0 = 0, ts1 = 0;
  uint32_t shard = wid % kQueueShards, tried = 0;" \
    kernels.hip "    if (!done && b0 < b1) {
      const bool phrase =" "    ts0 = __builtin_amdgcn_s_memrealtime();
    if (!done && b0 < b1) {
      const bool phrase =" \
    kernels.hip "    // The item's end from the events still in LDS where it can (finish_item
    // otherwise): every event of the item is there when ev_n == evb." "    ts1 = __builtin_amdgcn_s_memrealtime();
    t_seg += ts1 - ts0;" \
    kernels.hip "    item = 0xFFFFFFFFu;
  }
  if (fr.oj.nq > 0)" "    {
      const uint64_t te = __builtin_amdgcn_s_memrealtime();
      t_fin += te - ts1;
      t_fmax = te - ts1 > t_fmax ? te - ts1 : t_fmax;
    }
    item = 0xFFFFFFFFu;
  }
  if (fr.oj.nq > 0)" \
    kernels.hip "    stats[wid * kStatStride + 0] = n_surv;
    stats[wid * kStatStride + 1] = n_dblk;
    stats[wid * kStatStride + 2] = 0;" "    stats[wid * kStatStride + 0] = static_cast<uint32_t>(t_seg);
    stats[wid * kStatStride + 1] = n_dblk + 0u * n_surv;
    stats[wid * kStatStride + 2] = static_cast<uint32_t>(t_fin);
    stats[wid * kStatStride + 3] = static_cast<uint32_t>(t_fmax);"
  exit 0
fi
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p "$O"
# (--end: the endphase build of scripts/build_endphase.py, the item-end breakdown)
case "${2:-}" in
  --end) V=endphase; F=lean_endphase ;;
  --count) V=${3:-endcount}; F=lean_$V ;;   # (scripts/build_endcount.py [NAME ...])
  *) V=leanphase; F=lean_phase ;;
esac
WISER_HIP_LIB=$R/wiser_amd/_lib/variants/$V.so timeout -k 10 400 python3 scripts/lean_phase.py ${2:-} \
    > "$O/$F.json" 2> "$O/$F.err"
python3 - "$O/$F.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("alone", "pipelined"):
    for s in d[k][:4]:
        print(k, s)
PY
