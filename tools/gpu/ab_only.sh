#!/bin/bash
# A/B of ab/*.so on one config (no tests): bash tools/gpu/ab_only.sh <config>
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && bash tools/gpu/ab_libs.sh ${1:-2}
