#!/bin/bash
# B = 1 at 32 MiB/256: launch floor from C++, gf_gemv_kernel vs gf_gemm_kernel
# (events, interleaved) and their rocprofv3 kernel durations; parity of the
# gemv path first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-b1}; mkdir -p $OUT
KODR_GEMV=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "matmul or headline or encode or smoke or lazy_c2" --timeout 300 --timeout-method thread > $OUT/tests_gemv.log 2>&1 || { tail -30 $OUT/tests_gemv.log; exit 1; }
tail -1 $OUT/tests_gemv.log
timeout -k 10 120 tools/probe/launch_floor > $OUT/launch_floor.log 2>&1 || { cat $OUT/launch_floor.log; exit 1; }
cat $OUT/launch_floor.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/lf_trace -o lf -- tools/probe/launch_floor > $OUT/lf_trace.log 2>&1 || { tail -20 $OUT/lf_trace.log; exit 1; }
for rep in 1 2; do
  for G in 0 1; do
    KODR_GEMV=$G timeout -k 10 180 python -u tools/b1_ab.py > $OUT/gemv${G}_r$rep.log 2>&1 || { tail -20 $OUT/gemv${G}_r$rep.log; exit 1; }
    echo "gemv=$G rep $rep $(tail -1 $OUT/gemv${G}_r$rep.log)"
  done
done
for G in 0 1; do
  KODR_GEMV=$G timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_gemv$G -o run -- python3 tools/b1_ab.py > $OUT/prof_gemv$G.log 2>&1 || { tail -20 $OUT/prof_gemv$G.log; exit 1; }
done
find $OUT -name "*kernel_stats.csv" | head
