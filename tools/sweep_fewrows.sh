#!/bin/bash
# Few rows of X (K < 256) over wide rows: one-wave gf_gemm tiles vs the K-splitting ones (tools/tune_gemm.py).
set -e
for K in 32 64 128; do for L in 262144 1048576 4194304; do
  timeout -k 10 60 python tools/tune_gemm.py --M 1,4,8 --K $K --L $L --gens 4 --iters 50 --tiles "1,1,2;2,1,2;1,16,2;4,1,2;4,8,2;8,1,2;8,8,2;8,16,2" | sed "s/^/K=$K L=$L /"
done; done
