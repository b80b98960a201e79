#!/bin/bash
# round 3: config-4 tails on a stream of their own vs behind the small classes --
# records GPU tests + full-size config 4, a same-box A/B
# (ab/tails_stream.so, ab/tails_aux.so), then a kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py "tests/test_gpu_full_size.py::test_config4_full_size_zipf" \
    -x -q --timeout 400 --timeout-method thread > gpurun_out/r3_cfg4_tests.log 2>&1 || { tail -40 gpurun_out/r3_cfg4_tests.log; exit 1; }
tail -2 gpurun_out/r3_cfg4_tests.log
bash tools/gpu/ab_libs.sh 4 || exit 1
for n in tails_stream tails_aux; do
  rm -rf gpurun_out/prof_$n
  NOISE_AMD_LIB=$GRAFT_REPO_ROOT/ab/$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$n -o run -- \
      python3 bench.py --config 4 --steps 10 --no-cpu-baseline --no-config1 > gpurun_out/prof_$n.log 2>&1 || { tail -20 gpurun_out/prof_$n.log; exit 1; }
done
