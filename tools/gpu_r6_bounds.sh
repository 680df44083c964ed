#!/bin/bash
# Round 6, verdict item 2: the bit-sliced kernel's bounds at the round trip's
# shapes (B = 258: the encode's KW = 4 plan; B = 256: GetPieces' direct plan;
# B = 32 for reference), grouped launches over 16 prepared 32 MiB/256
# generations (tools/group_bs_time.py), in the tuning-modes build
# (kodr_amd/ab_modes, -DKODR_TUNE_MODES): MODE 0 the product loop, 30 every
# body inlined for one coefficient (no jumps, stubs or index mode; wrong
# products), 31 no row stream (stale rows), 32 neither.  Interleaved, MODE 0
# first and last.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r6_bounds; mkdir -p $O
for m in 0 30 31 32 0; do
  KODR_RLNC_LIB=kodr_amd/ab_modes/libkodr_rlnc.so KODR_BS_MODE=$m timeout -k 10 200 python -u tools/group_bs_time.py 258 256 32 \
    > $O/mode_$m.log 2>&1 || { echo "mode $m failed"; tail -5 $O/mode_$m.log; exit 1; }
  echo "mode $m: $(tail -1 $O/mode_$m.log | cut -c1-400)"
done
