#!/bin/bash
# round 4: what a live resident latency instance costs batch work on the same
# GPU.  Config-2 bench and the Pipeline 1 KiB bench, each alone, beside an
# idle (polling) instance and beside one under steady traffic (another
# process: transport_test resident_hold), alternating, twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/r4_resident_cost.txt
: > $OUT
bench() {  # $1 = label
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-config1 --steps 40 > gpurun_out/rc_b.json 2>/dev/null || return 1
  python3 -c "import json;d=json.load(open('gpurun_out/rc_b.json'));r=d['roofline'];print('$1 cfg2', d['value'], r['enc_ms'], r['dec_ms'])" >> $OUT
  timeout -k 10 120 noise-cpp_amd/bin/transport_test bench pipeline 1000 1048576 1024 8 > gpurun_out/rc_t.json 2>/dev/null || return 1
  python3 -c "import json;d=json.load(open('gpurun_out/rc_t.json'));print('$1 pipeline1k', d['encrypt_gib_s'], d['decrypt_gib_s'])" >> $OUT
}
for rep in 1 2; do
  bench alone || exit 1
  for busy in 0 1; do
    rm -f gpurun_out/rc_stop
    RESIDENT_HOLD_STOP=gpurun_out/rc_stop timeout -k 10 90 noise-cpp_amd/bin/transport_test resident_hold 60 $busy > gpurun_out/rc_hold_$busy.json &
    H=$!
    sleep 2
    bench resident_busy$busy; brc=$?
    touch gpurun_out/rc_stop; wait $H; hrc=$?
    cat gpurun_out/rc_hold_$busy.json >> $OUT
    [ $brc -eq 0 ] && [ $hrc -eq 0 ] || exit 1
  done
done
cat $OUT
