#!/bin/bash
# mc2 (the default for more than 7 decoders at k = 256) against mc4 with
# its per-launch cap raised (tuning build kodr_amd/tune_x: -DKODR_TUNE
# -DKODR_ELIM_MC_MAX_BLOCKS=1024, KODR_ELIM_MC=4) for G fresh k = 256
# decoders per batched GPU AddPiece (tools/elim_time.py), kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mc4_many; mkdir -p $O
G=${1:-16}
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/mc2 -o run --output-format csv -- \
  python3 tools/elim_time.py 256 $G 256 > $O/mc2.log 2>&1 &&
KODR_RLNC_LIB=kodr_amd/tune_x/libkodr_rlnc.so KODR_ELIM_MC=4 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
  -d $O/mc4 -o run --output-format csv -- python3 tools/elim_time.py 256 $G 256 > $O/mc4.log 2>&1
rc=$?
for v in mc2 mc4; do echo "== $v"; tail -3 $O/$v.log | cut -c1-300; grep -h "gf_elim" $O/$v/run_kernel_stats.csv | cut -c1-200; done
exit $rc
