#!/bin/bash
# A/B of gf_gemm tiles in three modes: 0 = normal, 1 = loads only (no GF
# arithmetic), 2 = arithmetic only (no loads).  Needs a KODR_TUNE_MODES build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for mode in 0 1 2; do
  KODR_GEMM_MODE=$mode timeout -k 10 120 python tools/tune_gemm.py --M 8 --tiles "8,16,2;4,8,2" --iters 200 | sed "s/^/mode=$mode /"
done
KODR_GEMM_MODE=0 timeout -k 10 120 python tools/tune_gemm.py --M 256 --tiles "8,4,1" --iters 20 | sed "s/^/mode=0 /"
KODR_GEMM_MODE=2 timeout -k 10 120 python tools/tune_gemm.py --M 256 --tiles "8,4,1" --iters 20 | sed "s/^/mode=2 /"
