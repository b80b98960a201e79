# X25519 + batched-handshake parity and throughput
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_x25519.py tests/test_gpu_handshake_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { tail -30 gpurun_out/pytest_x.log; exit 1; }
tail -2 gpurun_out/pytest_x.log
timeout -k 10 300 python tools/bench_x25519.py > gpurun_out/x25519.json && cat gpurun_out/x25519.json && timeout -k 10 300 python tools/bench_handshake.py 262144 XX IK NN XXpsk3 > gpurun_out/hs_bench.json && cat gpurun_out/hs_bench.json
