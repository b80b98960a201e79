set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for lib in r0 r1; do
  for L in 1024 4096; do
    NOISE_AMD_LIB=$R/ab/$lib.so timeout -k 10 120 python tools/bench_strided.py $L $((1048576 * 1024 / L)) 2>/dev/null | sed "s/^/$lib /" || exit 1
  done
done
done
