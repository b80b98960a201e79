#!/bin/bash
# round 4, final tree (nt DMA policy): gpu suite + smoke + bench, then the
# config-2 and config-4 rocprofv3 trace + PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/r4_final.sh || exit 1
rm -rf gpurun_out/prof_cfg2 gpurun_out/prof_cfg4
bash tools/gpu/profile_cfg.sh 2 20 || exit 1
bash tools/gpu/profile_cfg.sh 4 10
