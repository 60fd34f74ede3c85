#!/bin/bash
# PMC passes over the bench (one rocprofv3 process per pass; --pmc is never
# combined with sys/runtime traces).  Usage: scripts/profile_pmc.sh OUTDIR [bench args]
set -u
OUT=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$OUT/pass$i" -o pmc -- \
      python3 "$R/bench.py" --no-cpu --check 0 --steps 5 --warmup 1 "$@" > "$OUT/pass$i.json" 2> "$OUT/pass$i.err"
  rc=$?
  echo "pass $i ($counters): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum
LIST
