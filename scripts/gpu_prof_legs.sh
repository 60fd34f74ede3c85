#!/bin/bash
# Profiles of bench legs run alone (scripts/leg_run.py): kernel-trace stats,
# the batch overlap, and per-launch fabric bytes from three TCC_EA0 counter
# passes (scripts/pmc_bytes.py), for each leg named.  Every GPU step has its
# own limit; the first failure ends the script.  Usage: TAG LEG...  (c3 c4 c5)
set -eu -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_legprof_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd /tmp
for LEG in "$@"; do
  # index and log first, outside the profiler
  timeout -k 10 400 python3 "$R/scripts/leg_run.py" "$LEG" 1 > "$O/${LEG}_plain.json" 2> "$O/${LEG}_plain.err"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/$LEG/stats" -o stats -- \
      python3 "$R/scripts/leg_run.py" "$LEG" 8 > "$O/${LEG}_stats.json" 2> "$O/${LEG}_stats.err"
  find "$P/$LEG/stats" -name "*kernel_stats.csv" -exec cp {} "$O/${LEG}_kernel_stats.csv" \;
  find "$P/$LEG/stats" -name "*kernel_trace.csv" -exec cp {} "$P/${LEG}_trace.csv" \;
  python3 "$R/scripts/trace_overlap.py" "$P/${LEG}_trace.csv" > "$O/${LEG}_trace_overlap.json"
  echo "$LEG stats ok"
  i=0
  for counters in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE" \
                  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -k 10 400 rocprofv3 --pmc $counters --output-format csv -d "$P/$LEG/pmc/pass$i" -o pmc -- \
        python3 "$R/scripts/leg_run.py" "$LEG" 1 > "$O/${LEG}_pmc_pass$i.json" 2> "$O/${LEG}_pmc_pass$i.err"
    echo "$LEG pmc pass $i ok"
  done
  python3 "$R/scripts/pmc_bytes.py" "$P/$LEG/pmc" lean_kernel,segment_kernel "$O/${LEG}_pmc_segment.json" \
      "$O/${LEG}_pmc_pass1.json" > /dev/null
  python3 - "$O/${LEG}_pmc_segment.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], "bytes/launch", round(d["hbm_bytes_per_launch"] / 1e6, 1), "MB; algo",
      round(d.get("algo_bytes_per_launch", 0) / 1e6, 1), "MB; ratio", round(d.get("traffic_over_algo", 0), 3))
PY
done
