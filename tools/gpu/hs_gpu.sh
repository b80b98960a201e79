# batched-handshake GPU checks + bench: bash tools/gpu/hs_gpu.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_handshake_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hs_tests.log 2>&1 || { tail -40 gpurun_out/hs_tests.log; exit 1; }
tail -3 gpurun_out/hs_tests.log
timeout -k 10 300 python tools/bench_handshake.py 262144 XX IK NN XXpsk3 > gpurun_out/hs_bench.json && cat gpurun_out/hs_bench.json
