#!/bin/bash
# A round's GPU evidence in one call, each step time-limited and chained so
# the first failure ends it:
#   the -m gpu suite (one process) -> smoke() -> the default bench line (the
#   driver's command) -> rocprofv3 trace + PMC passes for the configs given
#   (default 2 and 4) -> gpurun_out/full_*, gpurun_out/prof_cfgN
# then on the CPU: python3 tools/gpu/summarize_cfg.py N roundNN
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --durations 10 > gpurun_out/full_tests.log 2>&1
rc=$?
tail -3 gpurun_out/full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err || { tail -20 gpurun_out/full_bench.err; exit 1; }
cat gpurun_out/full_bench.json
for c in ${@:-2 4}; do
  bash tools/gpu/profile_cfg.sh $c || exit 1
done
