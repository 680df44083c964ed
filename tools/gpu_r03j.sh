#!/bin/bash
# Recode with the vector columns as a side product spread over every
# workgroup of the bit-sliced launch: parity of the recode paths, interleaved
# timings against the separate vector launch (KODR_REC_SIDE=0), rocprof
# kernel durations of both at B = 32.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="$R/gpurun_out/${1:-r03j}"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_recode_side.py \
  tests/test_gpu_headline.py tests/test_gpu_compact.py tests/test_gpu_parity.py -k "recode or recoder" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for S in 1 0; do
    KODR_REC_SIDE=$S timeout -k 10 120 python -u tools/recode_time.py 9 16 32 64 256 > $OUT/rec_s${S}_r$rep.json 2>&1 || { tail -20 $OUT/rec_s${S}_r$rep.json; exit 1; }
    echo "side=$S rep $rep $(tail -1 $OUT/rec_s${S}_r$rep.json)"
  done
done
for S in 1 0; do
  KODR_REC_SIDE=$S timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_s$S" -o run -- \
    python3 "$R/tools/recode_time.py" 32 > "$OUT/prof_s$S.log" 2>&1 || { tail -20 "$OUT/prof_s$S.log"; exit 1; }
done
python3 "$R/tools/kernel_durations.py" "$OUT/prof_s1" "$OUT/prof_s0" | cut -c1-300
