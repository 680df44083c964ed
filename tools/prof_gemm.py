#!/usr/bin/env python3
"""Run one gf_gemm shape/tile N times (for rocprofv3 --pmc passes).
usage: KODR_GEMM_CFG=mt,kw,s python tools/prof_gemm.py M [iters] [K] [L]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors
from kodr_amd._lib import lib
M = int(sys.argv[1]); iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
K = int(sys.argv[3]) if len(sys.argv) > 3 else 256
L = int(sys.argv[4]) if len(sys.argv) > 4 else 131072
G = 16
ctx = device.Context(0)
rng = np.random.default_rng(0)
gen = ctx.alloc(G * K * L)
ctx.h2d(gen, rng.integers(0, 256, G * K * L, dtype=np.uint8))
dA = ctx.alloc(M * K); ctx.h2d(dA, rng.integers(0, 256, M * K, dtype=np.uint8))
dY = ctx.alloc(M * L)
for i in range(iters):
    errors.check(lib().rlnc_gf_matmul_device(ctx.handle, dA, K, M, K, gen + (i % G) * K * L, L, dY, L, L))
ctx.synchronize()
print("done", M, os.environ.get("KODR_GEMM_CFG"))
