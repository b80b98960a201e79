#!/bin/bash
# round 3: state of the tree -- full GPU suite, smoke, default bench, doorbell
# probe, config-1 per-record latency in both modes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
    --durations 10 > gpurun_out/r3_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { cat gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
cat gpurun_out/r3_bench.json
timeout -k 10 60 tools/ubench/doorbell_probe > gpurun_out/doorbell.txt 2>&1 || { cat gpurun_out/doorbell.txt; exit 1; }
cat gpurun_out/doorbell.txt
for m in launch resident; do
  timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 $m > gpurun_out/c1_$m.json 2>&1 || { cat gpurun_out/c1_$m.json; exit 1; }
  cat gpurun_out/c1_$m.json
done
timeout -k 10 60 tools/ubench/one_timing > gpurun_out/one_timing.txt 2>&1 && cat gpurun_out/one_timing.txt
