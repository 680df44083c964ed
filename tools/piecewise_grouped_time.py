"""C2 fed one AddPiece call per piece for 16 resident generations (bench.py
piecewise_grouped): the lazy queues flushed by one rlnc_decoders_flush_gpu
call against each decoder's own state read on the host.  usage: [G]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kodr_amd import device as kdev  # noqa: E402
from kodr_amd import errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
ctx = kdev.Context(0)
hs = bench.HeadlineStep(ctx, lib(), errors, bench.K_PIECES, bench.L_BYTES, 32, G, grouped=True,
                        rng=np.random.default_rng(1))
print(json.dumps(bench.piecewise_grouped(ctx, lib(), errors, hs.encs, bench.K_PIECES, bench.L_BYTES)), flush=True)
