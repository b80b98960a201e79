set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do timeout -k 10 120 python tools/gpu/dbg_segxor.py 4096 4096 | grep -E "segment|status" || exit 1; done
