#!/bin/bash
# One GPU-box session of round 3.  Steps (each GPU step under its own limit,
# the first failure ends the script):
#   tests   python -m pytest -m gpu, then smoke()
#   bench   the default bench line (C3 stand-in headline + every leg)
#   prof    kernel-trace stats + batch overlap of the headline workload, the EA
#           counter calibration, per-launch fabric bytes (PMC passes)
#   prof2   the same for the C2 leg (--workload c2)
# Usage: scripts/r03_gpu.sh TAG [tests] [bench] [prof] [prof2]   (default: all)
set -eu -o pipefail
TAG=$1; shift
STEPS=${*:-tests bench prof prof2}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=/tmp/wsr_prof_$TAG
mkdir -p "$O" "$P"
export TMPDIR=/tmp
has() { [[ " $STEPS " == *" $1 "* ]]; }

cd "$R"
if has tests; then
  timeout -k 10 1200 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
      > "$O/pytest_gpu.log" 2>&1
  tail -2 "$O/pytest_gpu.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
  echo "smoke ok"
fi
if has bench; then
  timeout -k 10 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
  echo "bench ok"; head -c 1500 "$O/bench.json"; echo
fi

prof() {   # $1 = workload key, $2... = extra bench args
  local wl=$1; shift
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/stats_$wl" -o stats -- \
      python3 "$R/bench.py" --no-cpu --no-extra --steps 2000 "$@" > "$O/bench_stats_$wl.json" 2> "$O/bench_stats_$wl.err"
  find "$P/stats_$wl" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_$wl.csv" \;
  find "$P/stats_$wl" -name "*kernel_trace.csv" -exec cp {} "$P/kernel_trace_$wl.csv" \;
  python3 "$R/scripts/trace_overlap.py" "$P/kernel_trace_$wl.csv" > "$O/trace_overlap_$wl.json"
  echo "stats $wl ok"
  local i=0
  for counters in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE" \
                  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    if [ "$wl" = c3 ]; then
      timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d "$P/calib/pass$i" -o pmc -- \
          "$R/wiser_amd/_lib/calib_ea" > "$O/calib_pass$i.json" 2> "$O/calib_pass$i.err"
    fi
    timeout -k 10 600 rocprofv3 --pmc $counters --output-format csv -d "$P/pmc_$wl/pass$i" -o pmc -- \
        python3 "$R/bench.py" --no-cpu --no-extra --check 0 --steps 25 --warmup 1 "$@" \
        > "$O/pmc_${wl}_pass$i.json" 2> "$O/pmc_${wl}_pass$i.err"
    echo "pmc $wl pass $i ok"
  done
  if [ "$wl" = c3 ]; then
    python3 "$R/scripts/pmc_bytes.py" "$P/calib" > "$O/calib_bytes.txt"
    cat "$O/calib_bytes.txt"
  fi
  python3 "$R/scripts/pmc_bytes.py" "$P/pmc_$wl" lean_kernel,segment_kernel "$O/pmc_segment_$wl.json" \
      "$O/pmc_${wl}_pass1.json" > /dev/null
  python3 "$R/scripts/pmc_bytes.py" "$P/pmc_$wl" > "$O/pmc_all_kernels_$wl.txt"
  cd "$R"
}
if has prof; then prof c3; fi
if has prof2; then prof c2 --workload c2; fi
echo done
