"""bench.RoundTripStep timed as bench.py times it (run_timed: warmup, barrier,
K steps, barrier) with the steps as they are ("async": the step returns while
GetPieces runs) and with a host wait at each step's end ("sync"),
interleaved.  usage: python tools/rt_variants.py [steps] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
L_ = lib()
ctx = kdev.Context(0)
k, L, G = 256, 131072, 16
hs = bench.HeadlineStep(ctx, L_, errors, k, L, 32, G, grouped=True, rng=np.random.default_rng(1))
rt = bench.RoundTripStep(ctx, L_, errors, hs.encs, k, L, np.random.default_rng(2))


def sync_step(i, timed=True):
    rt.step(i, timed)
    ctx.synchronize()


for rep in range(REPS):
    for name, fn in (("async", rt.step), ("sync", sync_step)):
        t, nw = bench.run_timed(fn, K, 5, ctx.synchronize, bench.WARM_S)
        print(f"rep {rep} {name:5s}: {t / K / G * 1e6:.2f} us/gen ({nw} warmup)", flush=True)
rt.close()
hs.close()
