#!/bin/bash
# Round 6: what the round trip's B = 258 encode pays for its last row group
# (2 real rows of 8): grouped launches over 16 prepared 32 MiB/256
# generations (tools/group_bs_time.py 258 256) in the tuning-modes build
# (kodr_amd/ab_modes): MODE 0 the product, MODE 38 the last partial row group
# skipped (wrong products); the encode's plan (KW = 4) and the direct plan
# (KODR_BS_KW=1); interleaved twice.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r6j; mkdir -p $O
for rep in 1 2; do
  for kw in 4 1; do
    for m in 0 38; do
      KODR_RLNC_LIB=kodr_amd/ab_modes/libkodr_rlnc.so KODR_BS_MODE=$m KODR_BS_KW=$kw timeout -k 10 200 \
        python -u tools/group_bs_time.py 258 256 > $O/m${m}_kw${kw}_$rep.log 2>&1 \
        || { echo "mode $m kw $kw failed"; tail -5 $O/m${m}_kw${kw}_$rep.log; exit 1; }
      echo "mode $m kw $kw rep $rep: $(tail -1 $O/m${m}_kw${kw}_$rep.log | cut -c1-300)"
    done
  done
done
