# kernel timeline of one bench config: bash tools/gpu/trace_cfg.sh <config>
set -o pipefail
R=$GRAFT_REPO_ROOT
C=${1:-4}
O=$R/gpurun_out/trace_cfg$C
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O -o trace --output-format csv -- python3 $R/bench.py --config $C --steps 3 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/err.log
