#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
B=noise-cpp_amd/bin/transport_test
for len in 256 1024; do timeout -k 10 200 $B bench pipeline 1000 1048576 $len 8 || exit 1; done
