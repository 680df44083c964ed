#!/bin/bash
# The batched elimination of 16 k = 256 decoders alone (L = 256) and with the
# round trip's piece length (L = 131,072: the row copies and twin beside it),
# GPU route vs host (tools/elim_time.py), with a kernel trace of both.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-elim_rt}; mkdir -p $OUT
R=$(pwd)
for L in 256 131072 131072s0; do
  S=1; [ "${L%s0}" != "$L" ] && { S=0; L=${L%s0}; }
  export KODR_ADD_SIDE=$S
  timeout -k 10 200 python -u tools/elim_time.py 256 ${GS:-16} $L > $OUT/e_L${L}_s$S.log 2>&1 || { tail -20 $OUT/e_L${L}_s$S.log; exit 1; }
  cat $OUT/e_L${L}_s$S.log
  cd /tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_L${L}_s$S -o run --output-format csv -- python3 $R/tools/elim_time.py 256 ${GS:-16} $L > $R/$OUT/prof_L${L}_s$S.log 2>&1 || { tail -20 $R/$OUT/prof_L${L}_s$S.log; exit 1; }
  cd $R
  python3 tools/kernel_durations.py $OUT/prof_L${L}_s$S 2>/dev/null | head -8 || true
done
