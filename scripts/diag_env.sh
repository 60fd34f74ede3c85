set -eu -o pipefail
cd $GRAFT_REPO_ROOT
for e in "X=1" "WSR_FUSE_REPLAY=0" "WSR_SEG_FLOOR=0" "WSR_DENSE_RATIO=0.5" "WSR_DENSE_DIV=64"; do
  echo "== $e"
  env $e timeout -k 10 300 python3 scripts/diag_types.py 2>&1 | grep -v "driver blocks"
done
