#!/bin/bash
# Fused replay (default) against the separate replay launch (WSR_FUSE_REPLAY=0)
# on the C2 main leg and the C3 stand-in leg.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for f in 1 0 1; do
  WSR_FUSE_REPLAY=$f timeout -k 10 600 python3 -u bench.py --no-cpu --legs c3_wiki_standin --steps 3000 \
      > "$O/fuse$f.json" 2> "$O/fuse$f.err"
  python3 -c "
import json;d=json.loads(open('$O/fuse$f.json').read().strip().splitlines()[-1]);r=d['roofline'];c=d['legs']['c3_wiki_standin']
print('fuse=$f C2', d['value'], d['ms_per_step'], r['avg_launch_ms'], d['p50_alone_ms'], '| C3', c['value'], c['segment_ms_per_batch'], c['p50_ms'])"
done
