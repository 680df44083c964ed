#!/bin/bash
# Round 6: B = 256 / 258 grouped launches alternated in one process (order
# check of tools/gpu_r6_j.sh), KW = 4, tuning-modes build, MODE 0 and 38.
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
for m in 0 38; do
  KODR_RLNC_LIB=kodr_amd/ab_modes/libkodr_rlnc.so KODR_BS_MODE=$m KODR_BS_KW=4 timeout -k 10 200 python -u tools/group_bs_time.py 256 258 256 258 > $O/order_m$m.log 2>&1 || exit 1
  echo "mode $m"; grep -v "^{" $O/order_m$m.log
done
