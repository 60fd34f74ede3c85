#!/bin/bash
# High x high class: fused replay against a separate replay launch
# (WSR_FUSE_REPLAY=0), and the end-of-item event re-filter left out.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for idx in c2 c3; do
  w=""
  [ $idx = c3 ] && w="--wiki"
  timeout -k 10 400 python3 scripts/diag_types.py $w --only high-high --repeat 3 > "$O/${idx}_default.txt" 2>&1
  echo "$idx default: $(grep -E '^high-high' "$O/${idx}_default.txt" | tail -1)"
  WSR_FUSE_REPLAY=0 timeout -k 10 400 python3 scripts/diag_types.py $w --only high-high --repeat 3 > "$O/${idx}_unfused.txt" 2>&1
  echo "$idx unfused: $(grep -E '^high-high' "$O/${idx}_unfused.txt" | tail -1)"
  WISER_HIP_LIB=$R/wiser_amd/_lib/var_norefilter/libwiser_hip.so timeout -k 10 400 python3 scripts/diag_types.py $w \
      --only high-high --repeat 3 > "$O/${idx}_norefilter.txt" 2>&1
  echo "$idx norefilter: $(grep -E '^high-high' "$O/${idx}_norefilter.txt" | tail -1)"
done
