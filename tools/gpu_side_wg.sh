#!/bin/bash
# the twin copy after the elimination (default) against beside it on the side
# stream at 4, 8 and 16 workgroups per CU (tuning build: KODR_ADD_SIDE=1,
# KODR_COPY_WG_PER_CU), the round trip timed as bench.py times it; then the
# timeline of the best side variant
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sidewg}; mkdir -p $OUT
T=kodr_amd/tune_c/libkodr_rlnc.so
for rep in 1 2; do
  echo "after: $(KODR_RLNC_LIB=$T timeout -k 10 200 python -u tools/rt_variants.py 20 1 2>&1 | grep async)"
  for n in 4 8 16; do
    echo "side wg $n: $(KODR_ADD_SIDE=1 KODR_COPY_WG_PER_CU=$n KODR_RLNC_LIB=$T timeout -k 10 200 python -u tools/rt_variants.py 20 1 2>&1 | grep async)"
  done
done
R=$(pwd)
cd /tmp
for n in 16 8; do
  KODR_ADD_SIDE=1 KODR_COPY_WG_PER_CU=$n KODR_RLNC_LIB=$R/$T timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tr_$n -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/tr_$n.json 2> $R/$OUT/tr_$n.err || { tail -20 $R/$OUT/tr_$n.err; exit 1; }
  echo "== side wg $n"; python3 $R/tools/rt_timeline.py $R/$OUT/tr_$n/run_kernel_trace.csv 3
done
