#!/bin/bash
# Round 6: the N > 1 bench path on one GPU -- the new tests (bench.py --gpus N
# spawning its own launcher, the deferred host replay taken by a phrase-only
# run), then an 8-rank gloo rehearsal of the whole N = 8 line through that
# spawn path.  Each GPU step has its own limit; the first
# failure ends the script.
set -eu -o pipefail
TAG=${1:-r06a}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_bench_multirank.py tests/test_shard_gpu.py -m gpu -x -v \
    --timeout 450 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
tail -3 "$O/pytest_gpu.log"
timeout -k 10 900 python3 bench.py --gpus 8 --exchange gloo --workload c2 --docs 200000 --vocab 100000 \
    --queries 40000 --steps 40 --warmup 4 --no-extra --no-cpu --check 128 --index-dir /tmp/wiser_n8 \
    > "$O/n8_gloo.json" 2> "$O/n8_gloo.err"
tail -c 1500 "$O/n8_gloo.json"
