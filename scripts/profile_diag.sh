#!/bin/bash
# PMC passes over scripts/diag_types.py (one query class).  Usage: OUTDIR CLASS
set -u
OUT=$1; CLS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/scripts/diag_types.py" --only "$CLS" > /dev/null 2>&1   # build index
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$OUT/pass$i" -o pmc -- \
      python3 "$R/scripts/diag_types.py" --only "$CLS" --repeat 3 > "$OUT/pass$i.txt" 2>&1
  rc=$?; echo "pass $i: rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH
SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_FLAT SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
FETCH_SIZE
LIST
python3 "$R/scripts/pmc_summary.py" "$OUT"
