#!/bin/bash
# round 4: what slows a Pipeline beside a resident instance of ANOTHER
# process?  Pipeline 1 KiB alone, beside a process with an idle HIP context
# only (hold 3), beside an idle polling instance (hold 2), beside one under a
# record every 5 ms (hold 0); alternating, three times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/r4_resident_cost2.txt
: > $OUT
pipe() {  # $1 = label
  timeout -k 10 120 noise-cpp_amd/bin/transport_test bench pipeline 1000 1048576 1024 8 > gpurun_out/rc2_t.json 2>/dev/null || return 1
  python3 -c "import json;d=json.load(open('gpurun_out/rc2_t.json'));print('$1 pipeline1k', d['encrypt_gib_s'], d['decrypt_gib_s'])" >> $OUT
}
for rep in 1 2 3; do
  pipe alone || exit 1
  for hold in 3 2 0; do
    rm -f gpurun_out/rc2_stop
    RESIDENT_HOLD_STOP=gpurun_out/rc2_stop timeout -k 10 90 noise-cpp_amd/bin/transport_test resident_hold 60 $hold > gpurun_out/rc2_hold_$hold.json &
    H=$!
    sleep 2
    pipe hold$hold; brc=$?
    touch gpurun_out/rc2_stop; wait $H; hrc=$?
    [ $brc -eq 0 ] && [ $hrc -eq 0 ] || { cat $OUT; exit 1; }
  done
done
cat $OUT
