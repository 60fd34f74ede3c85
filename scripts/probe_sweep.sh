#!/bin/bash
# Diagnostics only: scripts/probe_bench.hip over probe layouts, gaps, pool sizes.
# Usage: scripts/probe_sweep.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
B=$R/wiser_amd/_lib/probe_bench
for pool in 8192 2; do
  for gap in 183 60 500; do
    for layout in 0 1; do
      timeout -k 5 60 "$B" $layout $gap $pool 5 0 >> "$O/probe_sweep.jsonl"
    done
  done
done
for valu in 100 200; do
  for layout in 0 1; do
    timeout -k 5 60 "$B" $layout 183 8192 5 $valu >> "$O/probe_sweep.jsonl"
  done
done
for wgs in 2 8; do
  for layout in 0 1; do
    timeout -k 5 60 "$B" $layout 183 8192 $wgs 0 >> "$O/probe_sweep.jsonl"
  done
done
cat "$O/probe_sweep.jsonl"
