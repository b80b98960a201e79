#!/bin/bash
# round 5, first call: the -m gpu suite on the current tree, then the
# config-4 decrypt chunking / Poly1305-pass cache-policy A/B (ab/*.so,
# alternating, three rounds) -> gpurun_out/r5_call1_*
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --durations 10 > gpurun_out/r5_call1_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5_call1_tests.log
[ $rc -eq 0 ] || exit $rc
cp noise-cpp_amd/lib/libnoise_amd.so ab/c4nt.so
bash tools/gpu/ab_libs.sh 4 2>&1 | tee gpurun_out/r5_call1_cfg4_ab.txt
