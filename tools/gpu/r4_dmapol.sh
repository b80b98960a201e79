#!/bin/bash
# round 4: DMA cache policy variants (nt / sc1 nt / sc0 sc1 nt), configs 2 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for l in b_sc1 c_sc01; do
  NOISE_AMD_LIB=ab/$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q \
      --timeout 200 --timeout-method thread > gpurun_out/r4_dmapol_$l.log 2>&1 || { tail -30 gpurun_out/r4_dmapol_$l.log; exit 1; }
  tail -1 gpurun_out/r4_dmapol_$l.log
done
echo "== config 2"; bash tools/gpu/ab_libs.sh 2 || exit 1
echo "== config 4"; bash tools/gpu/ab_libs.sh 4
