#!/bin/bash
# Batched AddPiece wall time per call (tools/elim_time.py: G fresh decoders,
# GPU route vs kodr's elimination on the host) for the elimination kernels:
# KODR_ELIM_MC=0 (one workgroup per decoder), 2 (mc2), 4 (mc4), at several k
# and G.  Measurement only.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-modes}; mkdir -p $OUT
for rep in 1 2; do
  for M in ${MODES:-0 2 4}; do
    KODR_ELIM_MC=$M timeout -k 10 200 python -u tools/elim_time.py ${KS:-160,192,224,256} ${GS:-1,8,16} > $OUT/e_${M}_r$rep.log 2>&1 || { tail -20 $OUT/e_${M}_r$rep.log; exit 1; }
    echo "mc=$M rep $rep: $(python3 -c "import json,sys; print(' '.join(f\"k{d['k']}G{d['G']} {d['gpu_us']}/{d['host_us']}\" for d in map(json.loads, open(sys.argv[1]))))" $OUT/e_${M}_r$rep.log)"
  done
done
