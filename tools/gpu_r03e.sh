#!/bin/bash
# Round 3: recode with the vector columns as the bit-sliced launch's side
# product (and 3 body copies): its parity tests first, an interleaved A/B
# against the separate vector launch (KODR_REC_SIDE=0), then the full GPU
# suite, smoke, rocprof evidence of the headline and the driver's bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03e}; mkdir -p $OUT
timeout -k 10 60 tools/probe/cu_map 4096 > $OUT/cu_map.txt || exit 1
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_recode_side.py > $OUT/pytest_side.log 2>&1 || { tail -40 $OUT/pytest_side.log; exit 1; }
tail -1 $OUT/pytest_side.log
for rep in 1 2 3; do
  for S in 0 1; do
    KODR_REC_SIDE=$S timeout -k 10 120 python -u tools/recode_time.py > $OUT/rec_s${S}_r$rep.json 2>&1 || { tail -20 $OUT/rec_s${S}_r$rep.json; exit 1; }
    echo "side=$S rep $rep $(tail -1 $OUT/rec_s${S}_r$rep.json)"
  done
done
R="$(pwd)"
tools/pmc_icache.sh 32 "$R/kodr_amd/libkodr_rlnc.so" 0 c3 > $OUT/icache_c3.log 2>&1 || { tail -20 $OUT/icache_c3.log; exit 1; }
tools/pmc_icache.sh 32 "$R/kodr_amd/nc4/libkodr_rlnc.so" 0 c4 > $OUT/icache_c4.log 2>&1 || { tail -20 $OUT/icache_c4.log; exit 1; }
echo "icache 3 copies:"; cat $OUT/icache_c3.log; echo "icache 4 copies:"; cat $OUT/icache_c4.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
tools/profile_headline.sh || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['plan']); print(json.dumps(d['encode_decode'])[:400]); print(d['extras']['c2_decode']); print(d['extras']['c2_recode'])"
