#!/bin/bash
# Few rows of X over narrow rows (64-256 KiB): where the one-wave gf_gemm tiles stop paying (tools/tune_gemm.py).
set -e
for K in 16 32 64 128 200; do for L in 65536 131072 262144; do
  timeout -k 10 60 python tools/tune_gemm.py --M 1,2,4,8 --K $K --L $L --gens 8 --iters 50 --tiles "1,1,2;2,1,2;4,1,2;8,1,2;1,16,2;2,16,2;4,8,2;8,16,2" | sed "s/^/K=$K L=$L /"
done; done
