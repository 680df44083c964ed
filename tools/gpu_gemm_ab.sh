#!/bin/bash
# A/B of gf_gemm_kernel builds: kodr_amd/libkodr_rlnc.so (new) against
# kodr_amd/ab_old/libkodr_rlnc.so (old), both built beforehand on the CPU side.
# Parity tests of the new build first, then tune_gemm interleaved over builds.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="$R/gpurun_out/gemm_ab"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${AB_TESTS:-tests/test_gpu_parity.py} \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
  for v in new old; do
    LIB="$R/kodr_amd/libkodr_rlnc.so"; [ "$v" = old ] && LIB="$R/kodr_amd/ab_old/libkodr_rlnc.so"
    KODR_RLNC_LIB="$LIB" timeout -k 10 180 python -u tools/tune_gemm.py --M ${AB_M:-1,2,4,8} --tiles "${AB_TILES:-1,16,2;2,16,2;4,8,2;8,4,1}" --iters 200 \
      > "$OUT/${v}_r$rep.log" 2>&1 || { tail -20 "$OUT/${v}_r$rep.log"; exit 1; }
    sed "s/^/$v r$rep /" "$OUT/${v}_r$rep.log"
  done
done
