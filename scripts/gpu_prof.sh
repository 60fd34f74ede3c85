#!/bin/bash
# Profiles of the main C2 leg: kernel-trace stats, a kernel timeline (batch
# overlap), the EA counter calibration and per-launch fabric bytes.  Every GPU
# step has its own limit; the first failure ends the script.  Usage: TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_prof_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/stats" -o stats -- \
    python3 "$R/bench.py" --no-cpu --no-extra --steps 2000 > "$O/bench_stats.json" 2> "$O/bench_stats.err"
find "$P/stats" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
find "$P/stats" -name "*kernel_trace.csv" -exec cp {} "$P/kernel_trace.csv" \;
python3 "$R/scripts/trace_overlap.py" "$P/kernel_trace.csv" > "$O/trace_overlap.json"
echo "stats ok"
i=0
for counters in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE" \
                "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d "$P/calib/pass$i" -o pmc -- \
      "$R/wiser_amd/_lib/calib_ea" > "$O/calib_pass$i.json" 2> "$O/calib_pass$i.err"
  timeout -k 10 600 rocprofv3 --pmc $counters --output-format csv -d "$P/pmc/pass$i" -o pmc -- \
      python3 "$R/bench.py" --no-cpu --no-extra --check 0 --steps 5 --warmup 1 > "$O/pmc_pass$i.json" 2> "$O/pmc_pass$i.err"
  echo "pmc pass $i ok"
done
python3 "$R/scripts/pmc_bytes.py" "$P/calib" > "$O/calib_bytes.txt"
cat "$O/calib_bytes.txt"
python3 "$R/scripts/pmc_bytes.py" "$P/pmc" lean_kernel,segment_kernel "$O/pmc_segment.json" "$O/pmc_pass1.json"
python3 "$R/scripts/pmc_bytes.py" "$P/pmc" > "$O/pmc_all_kernels.txt"
echo done
# the sharded path rehearsed with one rank: where a step's time goes
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/shard" -o shard -- \
    python3 "$R/bench.py" --mode shard --no-cpu --no-extra --steps 300 > "$O/shard_stats.json" 2> "$O/shard_stats.err"
find "$P/shard" -name "*kernel_stats.csv" -exec cp {} "$O/shard_kernel_stats.csv" \;
echo "shard stats ok"
