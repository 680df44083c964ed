#!/bin/bash
# A/B of bit-sliced body alignment (gen_bs_bodies.py KODR_BS_ALIGN): builds
# kodr_amd/align{16,32}/libkodr_rlnc.so beforehand on the CPU side; here the
# headline-shape parity test under each variant, then tools/compact_time.py
# (compact encoder = bit-sliced kernel at every B) interleaved over variants.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="$R/gpurun_out/bs_align"; mkdir -p "$OUT"
for A in 16 32; do
  KODR_RLNC_LIB="$R/kodr_amd/align$A/libkodr_rlnc.so" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_compact.py tests/test_gpu_headline.py > "$OUT/tests_a$A.log" 2>&1 \
    || { tail -30 "$OUT/tests_a$A.log"; exit 1; }
  tail -1 "$OUT/tests_a$A.log"
done
for rep in 1 2; do
  for A in 0 16 32; do
    LIB="$R/kodr_amd/libkodr_rlnc.so"; [ "$A" != 0 ] && LIB="$R/kodr_amd/align$A/libkodr_rlnc.so"
    KODR_RLNC_LIB="$LIB" timeout -k 10 120 python -u tools/compact_time.py > "$OUT/t_a${A}_r$rep.json" 2>&1 \
      || { tail -20 "$OUT/t_a${A}_r$rep.json"; exit 1; }
    echo "align $A rep $rep $(cat "$OUT/t_a${A}_r$rep.json")"
  done
done
