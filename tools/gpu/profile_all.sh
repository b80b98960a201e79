#!/bin/bash
# rocprofv3 trace + PMC evidence for BASELINE configs 2..5 (tools/gpu/profile_cfg.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
for c in ${@:-2 3 4 5}; do
  bash $R/tools/gpu/profile_cfg.sh $c || exit 1
done
