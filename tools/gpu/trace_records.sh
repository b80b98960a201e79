# kernel timeline of tools/bench_records.py for given sizes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_records
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o trace --output-format csv -- python3 $R/tools/bench_records.py 1048576 4096 "$@" > $O/bench.json 2> $O/err.log
