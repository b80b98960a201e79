#!/bin/bash
# round 4: nt DMA policy, second same-box A/B (configs 2 and 4, 6 rounds each)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
echo "== config 2"; bash tools/gpu/ab_libs.sh 2 || exit 1; bash tools/gpu/ab_libs.sh 2 || exit 1
echo "== config 4"; bash tools/gpu/ab_libs.sh 4 || exit 1; bash tools/gpu/ab_libs.sh 4
