# transport pipeline parity + host-resident throughput (Batcher vs Pipeline,
# Pipeline with 1..16 copy threads)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "transport" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tr.log 2>&1 || { tail -30 gpurun_out/pytest_tr.log; exit 1; }
tail -2 gpurun_out/pytest_tr.log
B=noise-cpp_amd/bin/transport_test
timeout -k 10 200 $B bench batcher 1000 262144 1024 || exit 1
for t in 1 2 4 8 12; do timeout -k 10 200 $B bench pipeline 1000 1048576 1024 $t || exit 1; done
for t in 1 8; do timeout -k 10 200 $B bench pipeline 1000 1048576 256 $t || exit 1; done
for t in 1 8; do timeout -k 10 200 $B bench pipeline 100 65536 16384 $t || exit 1; done
