#!/bin/bash
# Round 6: the plan for the round trip's B = 258 encode, measured with the
# warm-up absorbed (tools/gpu_r6_l.sh): grouped launches over 16 prepared
# 32 MiB/256 generations (tools/group_bs_time.py 16 258 258 256 256, the
# first shape discarded) in a -DKODR_TUNE build (kodr_amd/ab_kw) with
# KODR_BS_KW = 4 (the planner's choice at 258), 1 (direct) and 8,
# interleaved three times.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/r6o; mkdir -p $O
for rep in 1 2 3; do
  for kw in 4 1 8; do
    KODR_RLNC_LIB=kodr_amd/ab_kw/libkodr_rlnc.so KODR_BS_KW=$kw timeout -k 10 200 \
      python -u tools/group_bs_time.py 16 258 258 256 256 > $O/kw${kw}_$rep.log 2>&1 || { echo "kw $kw failed"; exit 1; }
    echo "kw $kw rep $rep: $(grep -v '^{' $O/kw${kw}_$rep.log | awk '{print $1, $0}' | sed 's/single_us_per_generation/s/;s/grouped_us_per_generation/g/' | cut -c1-60 | tr '\n' ' ')"
  done
done
