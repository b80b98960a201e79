#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread \
    -k "resident or single or golden or kats or config1 or cipherstate or handshake_vectors" > gpurun_out/r3_res3_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3_res3_tests.log; exit 1; }
tail -2 gpurun_out/r3_res3_tests.log
for k in fine host; do timeout -k 10 60 tools/ubench/resident_timing $k > gpurun_out/restime_$k.txt 2>&1; rc=$?; cat gpurun_out/restime_$k.txt; [ $rc -eq 0 ] || exit $rc; done
for k in fine host; do
  NOISE_GPU_RESIDENT_REQ=$k timeout -k 10 120 noise-cpp_amd/bin/config1_bench 1000 1024 resident > gpurun_out/c1_res_$k.json 2>&1 || { cat gpurun_out/c1_res_$k.json; exit 1; }
  echo "$k: $(cat gpurun_out/c1_res_$k.json)"
done
