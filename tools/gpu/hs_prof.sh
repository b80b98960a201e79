# rocprofv3 kernel stats + one PMC pass of the batched XX handshake bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hs_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o hs --output-format csv -- $R/noise-cpp_amd/bin/handshake_test batch_bench XX 262144 1 > $O/bench_trace.json 2> $O/trace.err || exit 1
echo trace ok
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc -o pmc --output-format csv -- $R/noise-cpp_amd/bin/handshake_test batch_bench XX 262144 1 > $O/bench_pmc.json 2> $O/pmc.err || exit 1
echo pmc ok
