#!/bin/bash
# Last GPU call of the session: parity suite, smoke, the default bench line,
# the driver's short form, then the C3 kernel-trace stats and PMC traffic.
set -eu -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
bash scripts/r03_final.sh "$TAG" tests bench driver
bash scripts/r03_gpu.sh "$TAG" prof
