#!/bin/bash
# GPU tests of the current build, then A/B of ab/*.so on a config, then the VALU probes
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-2}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu/ab_libs.sh $C || exit 1
if [ -x tools/ubench/valu_classes ]; then timeout -k 10 120 tools/ubench/valu_classes > gpurun_out/valu_classes2.txt 2>&1 || exit 1; fi
