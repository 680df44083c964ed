#!/bin/bash
# Body alignment re-measured with 3 body copies (48 KB packed: aligned copies
# now fit the instruction cache): kodr_amd/{a16,a32,n2a32}/libkodr_rlnc.so
# built beforehand (KODR_BS_ALIGN 16 / 32 with 3 copies, 32 with 2 copies).
# Parity of the bit-sliced paths under each, then grouped and single-launch
# timings interleaved with the shipped build.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="$R/gpurun_out/${1:-align3_ab}"; mkdir -p "$OUT"
lib() { if [ "$1" = base ]; then echo "$R/kodr_amd/libkodr_rlnc.so"; else echo "$R/kodr_amd/$1/libkodr_rlnc.so"; fi; }
for V in a16 a32 n2a32; do
  KODR_RLNC_LIB="$(lib $V)" timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
    tests/test_gpu_headline.py tests/test_gpu_compact.py > "$OUT/tests_$V.log" 2>&1 || { tail -30 "$OUT/tests_$V.log"; exit 1; }
  echo "$V: $(tail -1 "$OUT/tests_$V.log")"
done
for rep in 1 2 3; do
  for V in base a16 a32 n2a32; do
    KODR_RLNC_LIB="$(lib $V)" timeout -k 10 180 python -u tools/group_bs_time.py 16 32 64 256 > "$OUT/g_${V}_r$rep.log" 2>&1 \
      || { tail -20 "$OUT/g_${V}_r$rep.log"; exit 1; }
    echo "$V rep $rep grouped $(python3 -c "import json; d=json.loads(open('$OUT/g_${V}_r$rep.log').read().strip().splitlines()[-1]); print([d[k]['grouped_us_per_generation'] for k in ('B16','B32','B64','B256')])")"
  done
done
