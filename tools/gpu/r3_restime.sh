#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for k in fine host; do timeout -k 10 60 tools/ubench/resident_timing $k > gpurun_out/restime_$k.txt 2>&1; rc=$?; cat gpurun_out/restime_$k.txt; [ $rc -eq 0 ] || exit $rc; done
