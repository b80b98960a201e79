#!/bin/bash
# round 4: config-1 latency A/B (round-3 library vs this tree), then the
# cost of a live resident instance to batch work
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu/ab_config1.sh > gpurun_out/r4_c1_ab.txt 2>&1 || { cat gpurun_out/r4_c1_ab.txt; exit 1; }
cat gpurun_out/r4_c1_ab.txt
bash tools/gpu/r4_resident_cost.sh
