#!/bin/bash
# One GPU-box session: parity tests, smoke, default bench, kernel-trace stats,
# PMC traffic passes.  Every GPU step has its own time limit; the first failure
# ends the script.  Raw rocprofv3 output stays in /tmp on the box; only the
# summaries land in gpurun_out/TAG.  Usage: scripts/round_gpu.sh TAG
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_prof_$TAG
mkdir -p "$O" "$P"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
echo "pytest gpu ok"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
echo "smoke ok"
timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
cd /tmp
# the main leg only (--no-extra): the per-kernel averages are those of the C2 batches
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/stats" -o stats -- \
    python3 "$R/bench.py" --no-cpu --no-extra > "$O/bench_stats.json" 2> "$O/bench_stats.err"
find "$P/stats" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
echo "stats ok"
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $counters --output-format csv -d "$P/pmc/pass$i" -o pmc -- \
      python3 "$R/bench.py" --no-cpu --no-extra --check 0 --steps 5 --warmup 1 > "$O/pmc_pass$i.json" 2> "$O/pmc_pass$i.err"
  echo "pmc pass $i ok"
done
python3 "$R/scripts/pmc_traffic.py" "$P/pmc" lean_kernel,segment_kernel "$O/pmc_segment.json"
echo done
