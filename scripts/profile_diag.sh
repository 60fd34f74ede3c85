#!/bin/bash
# PMC passes over scripts/diag_types.py (one query class), one rocprofv3
# process per pass (--pmc is never combined with sys/runtime traces).
# Usage: OUTDIR CLASS [COUNTER_FILE]   (one pass per line of COUNTER_FILE)
set -u
OUT=$(realpath -m "$1"); CLS=$2; LISTF=${3:+$(realpath "$3")}
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/scripts/diag_types.py" --only "$CLS" > /dev/null 2>&1   # build index
if [ -z "$LISTF" ]; then
  LISTF=$OUT/counters.txt
  cat > "$LISTF" <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH
FETCH_SIZE
LIST
fi
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$OUT/pass$i" -o pmc -- \
      python3 "$R/scripts/diag_types.py" --only "$CLS" --repeat 3 > "$OUT/pass$i.txt" 2>&1
  rc=$?; echo "pass $i: rc=$rc"; [ $rc -eq 0 ] || exit $rc
done < "$LISTF"
python3 "$R/scripts/pmc_summary.py" "$OUT"
