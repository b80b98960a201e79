# records tests, then config-4 A/B of ab/*.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mixed.log 2>&1 || { tail -30 gpurun_out/pytest_mixed.log; exit 1; }
tail -2 gpurun_out/pytest_mixed.log
bash tools/gpu/ab_libs.sh 4
