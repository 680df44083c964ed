#!/bin/bash
# Batched GPU AddPiece + grouped GetPieces over 16 fresh 32 MiB/256 decoders:
# row copies on a side stream beside the elimination (KODR_ADD_SIDE=1) or
# before it (0); per-decoder host work on 1 or 8 host threads
# (KODR_HOST_THREADS).  Parity first, then the bench's encode_decode legs,
# interleaved; phase times of one AddPiece call (KODR_ADD_TIMING=1).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-add_ab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_group_decode.py tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2 3; do
  for V in "0 1" "1 1" "1 8"; do
    set -- $V
    KODR_ADD_SIDE=$1 KODR_HOST_THREADS=$2 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline > $OUT/b_s$1_t$2_r$rep.json 2> $OUT/b_s$1_t$2_r$rep.err || { tail -20 $OUT/b_s$1_t$2_r$rep.err; exit 1; }
    python3 -c "import json,sys; e=json.load(open('$OUT/b_s$1_t$2_r$rep.json'))['encode_decode']; print('side=$1 threads=$2 rep $rep', {k: e[k] for k in ('us_per_generation','encode_us_per_generation','add_us_per_generation','get_us_per_generation','roundtrip_ok')})"
  done
done
KODR_ADD_TIMING=1 timeout -k 10 120 python -u tools/group_add_time.py 16 > $OUT/t_timing.log 2>&1 || { tail -20 $OUT/t_timing.log; exit 1; }
grep add_pieces_gpu $OUT/t_timing.log | tail -3; tail -1 $OUT/t_timing.log
