#!/bin/bash
# round 3: full GPU suite, smoke, config-1 both modes, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    --durations 5 > gpurun_out/r3_full_tests.log 2>&1 || { tail -40 gpurun_out/r3_full_tests.log; exit 1; }
tail -2 gpurun_out/r3_full_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { cat gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
for m in resident launch; do
  timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 $m > gpurun_out/c1_$m.json 2>&1 || { cat gpurun_out/c1_$m.json; exit 1; }
  echo "$m: $(cat gpurun_out/c1_$m.json)"
done
timeout -k 10 400 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
cat gpurun_out/r3_bench.json
