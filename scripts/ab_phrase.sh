#!/bin/bash
# A/B of the phrase leg (c5_phrase) and the main value: default build and every
# variant build (make variant V=... F=...), twice, on one box.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
run() {
  timeout -k 10 300 python3 bench.py --no-cpu --steps 10 --warmup 2 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());c=d['legs']['c5_phrase'];print('value', d['value'], 'mixed', d['legs']['c4_mixed_1to5']['value'], d['legs']['c4_mixed_1to5']['segment_ms_per_batch'], 'phrase', c['value'], 'phrase_seg', c['segment_ms_per_batch'])"
}
for round in 1 2; do
  echo "== default ($round)"; run
  for d in wiser_amd/_lib/var_*/; do
    echo "== $(basename $d) ($round)"
    WISER_HIP_LIB=$R/$d/libwiser_hip.so run
  done
done
