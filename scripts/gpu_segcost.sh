#!/bin/bash
# C2 main leg with the work-item size variants (make variant V=seg32 / seg16):
# throughput, isolated launch time, p50 of one batch alone.  Usage: TAG [variants]
set -eu -o pipefail
TAG=$1
shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for v in default "$@"; do
  lib=""
  [ "$v" != default ] && lib="$R/wiser_amd/_lib/var_$v/libwiser_hip.so"
  WISER_HIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra --steps 3000 \
      > "$O/$v.json" 2> "$O/$v.err"
  echo "$v $(python3 -c "import json;d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d['p50_alone_ms'])")"
done
