#!/bin/bash
# Fixed vs per-row cost of gf_gemm: time M=8 at K = 256/512/1024 in normal and
# compute-only modes (needs a KODR_TUNE_MODES build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for K in 256 512 1024; do
  for mode in 0 2; do
    KODR_GEMM_MODE=$mode timeout -k 10 120 python tools/tune_gemm.py --M 8 --K $K --L 65536 --gens 8 --iters 100 --tiles "8,16,2,2" | sed "s/^/K=$K mode=$mode /"
  done
done
