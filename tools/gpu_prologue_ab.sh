#!/bin/bash
# Bit-sliced prologue: every program coefficient loaded ahead of the row ring
# (new, kodr_amd/libkodr_rlnc.so) against 8 per lane per round (old build in
# kodr_amd/ab_old/): parity on the new build, then interleaved grouped
# timings (tools/group_bs_time.py) and the headline step (bench.py --no-extras).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prologue_ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_group_wire.py tests/test_gpu_compact.py tests/test_gpu_recode_side.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2 3; do
  for V in old new; do
    LIB=kodr_amd/libkodr_rlnc.so; [ $V = old ] && LIB=kodr_amd/ab_old/libkodr_rlnc.so
    KODR_RLNC_LIB=$LIB timeout -k 10 150 python -u tools/group_bs_time.py 32 256 > $OUT/g_${V}_r$rep.log 2>&1 || { tail -20 $OUT/g_${V}_r$rep.log; exit 1; }
    KODR_RLNC_LIB=$LIB timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-encode-decode > $OUT/b_${V}_r$rep.json 2> $OUT/b_${V}_r$rep.err || { tail -20 $OUT/b_${V}_r$rep.err; exit 1; }
    echo "$V rep $rep: $(head -2 $OUT/g_${V}_r$rep.log | tr '\n' ' ') | headline $(python3 -c "import json; d=json.load(open('$OUT/b_${V}_r$rep.json')); print(d['value'], d['roofline']['avg_launch_us'])")"
  done
done
