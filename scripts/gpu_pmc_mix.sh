#!/bin/bash
# Instruction mix, wait and memory-pipeline counters of bench legs run alone
# (scripts/leg_run.py, one pass over the leg's batches), one rocprofv3 pass per
# counter line of scripts/counters_hh.txt, summed per kernel by
# scripts/pmc_summary.py.  Every GPU step has its own limit; the first failure
# ends the script.  Usage: TAG LEG...
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for LEG in "$@"; do
  P=/tmp/wsr_pmcmix_${TAG}_$LEG
  mkdir -p "$P"
  timeout -k 10 400 python3 "$R/scripts/leg_run.py" "$LEG" 1 > "$O/${LEG}_mix_plain.json" 2> "$O/${LEG}_mix_plain.err"
  i=0
  while read -r counters; do
    [ -z "$counters" ] && continue
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d "$P/pass$i" -o pmc -- \
        python3 "$R/scripts/leg_run.py" "$LEG" 1 > "$O/${LEG}_mix_pass$i.json" 2> "$O/${LEG}_mix_pass$i.err" \
        && echo "$LEG pass $i ok" || { echo "$LEG pass $i failed: $counters"; tail -3 "$O/${LEG}_mix_pass$i.err"; exit 1; }
  done < "$R/scripts/counters_hh.txt"
  python3 "$R/scripts/pmc_summary.py" "$P" > "$O/${LEG}_pmc_mix.json"
done
