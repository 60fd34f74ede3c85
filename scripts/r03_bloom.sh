#!/bin/bash
# Phrase bloom pruning on the GPU: parity (phrase tests incl. the tampered-
# filter test, reference KATs), then the bloom_factor 0 / 1 A/B.  Usage: TAG [n_docs]
set -eu -o pipefail
TAG=$1
N=${2:-200000}
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_phrase.py tests/test_gpu_kats.py -x -v \
    --timeout 300 --timeout-method thread > "$O/pytest_phrase.log" 2>&1
tail -2 "$O/pytest_phrase.log"
timeout -k 10 900 python3 scripts/phrase_bloom_ab.py /tmp/wsr_bloom_ab "$N" 8192 > "$O/bloom_ab.json" 2> "$O/bloom_ab.err"
tail -5 "$O/bloom_ab.err"
