#!/bin/bash
# Quick gf_elim_mc2_kernel variant check: the elimination/decode parity tests
# under KODR_MC2_VARIANT=$V, one and 16 decoders' batched AddPiece for the
# variants in CONFIGS (mc:variant), and the tuning build's timeline of one
# decoder under $V (tools/elim_mc2_timing.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mc2v}; mkdir -p $OUT
V=${V:-4}
KODR_MC2_VARIANT=$V KODR_ROUTE_MIN_K=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests (variant $V) $(tail -1 $OUT/tests.log)"
for rep in 1 2; do
  for C in ${CONFIGS:-"2:0 2:$V"}; do
    M=${C%%:*}; W=${C##*:}
    KODR_ELIM_MC=$M KODR_MC2_VARIANT=$W timeout -k 10 120 python -u tools/elim_time.py 128,256 1,16 > $OUT/e_${M}_${W}_r$rep.log 2>&1 || { tail -20 $OUT/e_${M}_${W}_r$rep.log; exit 1; }
    echo "mc=$M var=$W rep $rep: $(python3 -c "import json,sys; print(' '.join(f\"k{d['k']}G{d['G']} {d['gpu_us']}/{d['host_us']}\" for d in map(json.loads, open(sys.argv[1]))))" $OUT/e_${M}_${W}_r$rep.log)"
  done
done
KODR_MC2_VARIANT=$V KODR_RLNC_LIB=kodr_amd/tune_e/libkodr_rlnc.so KODR_ELIM_DUMP=/tmp/mc2_dump_1.bin timeout -k 10 60 python -u tools/elim_mc2_timing.py 256 1 > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
tail -3 $OUT/phases.log
