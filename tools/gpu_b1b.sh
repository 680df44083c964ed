#!/bin/bash
# gf_gemv_kernel with precomputed register tables, 2 or 4 lane groups, against
# gf_gemm_kernel at B = 1 (events, interleaved) + rocprof durations; grouped
# headline step with 32 instead of 16 generations.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-b1b}; mkdir -p $OUT
for G in 2 4; do
  KODR_GEMV=$G timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "matmul or encode_vs or headline_launch or c2_roundtrip" --timeout 300 --timeout-method thread > $OUT/tests_gemv$G.log 2>&1 || { tail -30 $OUT/tests_gemv$G.log; exit 1; }
  tail -1 $OUT/tests_gemv$G.log
done
for rep in 1 2; do
  for G in 0 2 4; do
    KODR_GEMV=$G timeout -k 10 180 python -u tools/b1_ab.py > $OUT/gemv${G}_r$rep.log 2>&1 || { tail -20 $OUT/gemv${G}_r$rep.log; exit 1; }
    echo "gemv=$G rep $rep $(tail -1 $OUT/gemv${G}_r$rep.log)"
  done
done
for G in 2 4; do
  KODR_GEMV=$G timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_gemv$G -o run -- python3 tools/b1_ab.py > $OUT/prof_gemv$G.log 2>&1 || { tail -20 $OUT/prof_gemv$G.log; exit 1; }
done
for GG in 16 32; do
  KODR_GROUP_G=$GG timeout -k 10 180 python -u tools/group_bs_time.py 32 > $OUT/group_G$GG.log 2>&1 || { tail -20 $OUT/group_G$GG.log; exit 1; }
  echo "G=$GG $(tail -1 $OUT/group_G$GG.log)"
done
