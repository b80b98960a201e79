#!/bin/bash
# round 4: the sharded bench path with every rank's whole shard checked
# against the oracle (bench.py --check-oracle), configs 2 / 5 / 4 at 2 ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 400 \
    --timeout-method thread --durations 10 > gpurun_out/r4_multirank.log 2>&1
rc=$?
tail -20 gpurun_out/r4_multirank.log
exit $rc
