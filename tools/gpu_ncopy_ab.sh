#!/bin/bash
# A/B of the bit-sliced body copy count (gen_bs_bodies.py KODR_BS_NCOPY):
# kodr_amd/nc{3,2}/libkodr_rlnc.so are built beforehand on the CPU side.
# Parity of the bit-sliced paths under each variant, then grouped and single
# launch timings interleaved over variants (4 copies = the shipped build).
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="$R/gpurun_out/${1:-ncopy_ab}"; mkdir -p "$OUT"
lib() { if [ "$1" = 4 ]; then echo "$R/kodr_amd/libkodr_rlnc.so"; else echo "$R/kodr_amd/nc$1/libkodr_rlnc.so"; fi; }
for C in 3 2; do
  KODR_RLNC_LIB="$(lib $C)" timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
    tests/test_gpu_headline.py tests/test_gpu_compact.py tests/test_gpu_group_wire.py > "$OUT/tests_c$C.log" 2>&1 \
    || { tail -30 "$OUT/tests_c$C.log"; exit 1; }
  echo "ncopy $C: $(tail -1 "$OUT/tests_c$C.log")"
done
for rep in 1 2 3; do
  for C in 4 3 2; do
    KODR_RLNC_LIB="$(lib $C)" timeout -k 10 180 python -u tools/group_bs_time.py 16 32 64 256 > "$OUT/g_c${C}_r$rep.log" 2>&1 \
      || { tail -20 "$OUT/g_c${C}_r$rep.log"; exit 1; }
    echo "ncopy=$C rep $rep grouped $(python3 -c "import json; d=json.loads(open('$OUT/g_c${C}_r$rep.log').read().strip().splitlines()[-1]); print([d[k]['grouped_us_per_generation'] for k in ('B16','B32','B64','B256')])")"
    KODR_RLNC_LIB="$(lib $C)" timeout -k 10 120 python -u tools/compact_time.py > "$OUT/s_c${C}_r$rep.json" 2>&1 \
      || { tail -20 "$OUT/s_c${C}_r$rep.json"; exit 1; }
    echo "ncopy=$C rep $rep single $(tail -1 "$OUT/s_c${C}_r$rep.json")"
  done
done
