#!/bin/bash
# Round 6 final profiles, part 2: the C4, C5, single_high and realistic_mix
# legs (scripts/gpu_prof_legs.sh), then the kernel-trace summary of bench.py's
# own headline in the driver's form, then bench.py in the driver's form with
# every leg (traffic attached from these profiles).  Each GPU step has its
# own limit; the first failure ends the script.
set -eu -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06p
mkdir -p "$O"
cd "$R"
bash scripts/gpu_prof_legs.sh r06p c4_mixed_1to5 c5_phrase single_high realistic_mix
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/wsr_benchprof -o bench -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-extra --no-cpu > "$O/bench_under_rocprof.json" 2> "$O/bench_under_rocprof.err"
find /tmp/wsr_benchprof -name "*kernel_stats.csv" -exec cp {} "$O/bench_kernel_stats.csv" \;
echo "bench under rocprof ok"
