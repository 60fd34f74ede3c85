#!/bin/bash
# Diagnostics only: probe element forms (scripts/probe_bench.hip FORM) at the
# C3 gap from an 8 GB pool, and the EA request sizes of forms 0, 3, 4.
# Usage: scripts/probe_sweep2.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
B=$R/wiser_amd/_lib/probe_bench
for gap in 183 60; do
  for form in 0 1 2 3 4; do
    timeout -k 5 60 "$B" 0 $gap 8192 5 0 $form >> "$O/probe_forms.jsonl"
  done
done
cd /tmp
export TMPDIR=/tmp
for form in 0 3 4; do
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum \
      --output-format csv -d /tmp/pb_pmc_$form -o pmc -- "$B" 0 183 8192 5 0 $form > /dev/null 2>&1
  f=$(find /tmp/pb_pmc_$form -name "*counter_collection.csv" | head -1)
  echo "form $form: $(python3 -c "
import csv,sys,collections
s=collections.Counter()
for r in csv.DictReader(open('$f')): s[r['Counter_Name']]+=float(r['Counter_Value'])
print(dict(s))")" >> "$O/probe_forms_pmc.txt"
done
cat "$O/probe_forms.jsonl" "$O/probe_forms_pmc.txt"
