#!/bin/bash
# Many decoders per elimination launch at k = 256 (tools/elim_time.py, kernel
# trace of each): the shipped library (mc4 for one decoder, mc2 for 16)
# against the tuning build kodr_amd/tune_x (-DKODR_TUNE
# -DKODR_ELIM_MC_MAX_BLOCKS=1024 -DKODR_MC_PROBE=1: mc4's hand-off waits probe
# one granule between full polls) with KODR_ELIM_MC=4 (mc4 for 16 too).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mc4_many; mkdir -p $O
T=kodr_amd/tune_x/libkodr_rlnc.so
run() {  # name, lib, mc mode, G
  KODR_RLNC_LIB=$2 KODR_ELIM_MC=$3 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$1 -o run \
    --output-format csv -- python3 tools/elim_time.py 256 $4 256 > $O/$1.log 2>&1
}
run base_g1 kodr_amd/libkodr_rlnc.so 3 1 && run probe_g1 $T 3 1 &&
run base_g16 kodr_amd/libkodr_rlnc.so 3 16 && run probe_g16_mc4 $T 4 16 && run probe_g16_mc2 $T 2 16 &&
run base_g8 kodr_amd/libkodr_rlnc.so 3 8 && run probe_g8_mc4 $T 4 8
rc=$?
for v in base_g1 probe_g1 base_g16 probe_g16_mc4 probe_g16_mc2 base_g8 probe_g8_mc4; do
  echo "== $v $(grep '^{' $O/$v.log | cut -c1-200)"; grep -h "gf_elim" $O/$v/run_kernel_stats.csv | cut -d, -f1-7 | cut -c1-220
done
exit $rc
