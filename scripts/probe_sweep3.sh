#!/bin/bash
# Diagnostics only: two-level probes (scripts/probe_bench2.hip) against one level.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
B=$R/wiser_amd/_lib/probe_bench2
for rho in 0.005 0.01 0.02 0.05; do
  for g in 0 2 4 8 16; do
    timeout -k 5 60 "$B" 183 $rho $g 8192 5 >> "$O/probe_2level.jsonl"
  done
done
cat "$O/probe_2level.jsonl"
