#!/bin/bash
# Round 6: waves per workgroup (KW) at the round trip's encode shape, B = 258
# (and 256), grouped over 16 prepared 32 MiB/256 generations
# (tools/group_bs_time.py), tuning build kodr_amd/ab_modes: KODR_BS_KW forces
# the plan's KW (1 = direct), KODR_SPLIT_TAIL=0; interleaved twice.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r6_kw; mkdir -p $O
for rep in 1 2; do
  for kw in 4 2 3 1 8; do
    KODR_RLNC_LIB=kodr_amd/ab_modes/libkodr_rlnc.so KODR_SPLIT_TAIL=0 KODR_BS_KW=$kw timeout -k 10 200 \
      python -u tools/group_bs_time.py 258 256 > $O/kw_${kw}_$rep.log 2>&1 || { echo "kw $kw failed"; tail -5 $O/kw_${kw}_$rep.log; exit 1; }
    echo "kw $kw rep $rep: $(tail -1 $O/kw_${kw}_$rep.log | cut -c1-300)"
  done
done
