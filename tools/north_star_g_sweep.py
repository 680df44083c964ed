"""North-star shape (one coded piece per resident 32 MiB/256 generation per
grouped launch, bench.py grouped_encode) over G = 16, 32, 64 generations
per launch: HBM fraction of the generation reads.  usage: [G ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kodr_amd import device as kdev  # noqa: E402
from kodr_amd import errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

ctx = kdev.Context(0)
Gs = [int(x) for x in sys.argv[1:]] or [16, 32, 64]
hs = bench.HeadlineStep(ctx, lib(), errors, bench.K_PIECES, bench.L_BYTES, 32, max(Gs), grouped=True,
                        rng=np.random.default_rng(2))
for G in Gs:
    r = bench.grouped_encode(ctx, lib(), errors, hs.encs[:G], bench.K_PIECES, bench.L_BYTES,
                             np.random.default_rng(3))
    print(json.dumps({"G": G, "1": r["1"], "2": r["2"]}), flush=True)
