set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $R/gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> $R/gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > $R/gpurun_out/bench.json 2> $R/gpurun_out/bench.err || exit 1
