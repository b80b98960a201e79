#!/bin/bash
# round 4: the whole -m gpu suite (one pytest process), then the config-1
# latency leg (resident / launch) as a quick check of the single-record path
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r4}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    --durations 15 > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 1 > gpurun_out/${TAG}_config1.json 2>gpurun_out/${TAG}_config1.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_config1.json'));print({k: d[k].get('per_record') for k in ('build','build_launch')})"
