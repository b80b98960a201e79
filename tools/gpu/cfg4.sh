set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_mixed.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mixed.log 2>&1 || { tail -30 gpurun_out/pytest_mixed.log; exit 1; }
tail -2 gpurun_out/pytest_mixed.log
for i in 1 2; do timeout -k 10 300 python bench.py --config 4 --steps 5 --no-cpu-baseline > gpurun_out/cfg4_$i.json && python -c "import json;d=json.load(open('gpurun_out/cfg4_$i.json'));print('cfg4',d['value'],d['roofline']['enc_ms'],d['roofline']['dec_ms'])" || exit 1; done
