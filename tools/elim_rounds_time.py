"""Batched AddPiece over G decoders fed in several rounds (bench.py
batched_elim_rounds): host elimination per decoder against one
rlnc_decoders_add_pieces_gpu call per round, where every round after the
first runs on continued decoders.  usage: elim_rounds_time.py [k G rounds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kodr_amd import device as kdev  # noqa: E402
from kodr_amd import errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

k, G, rounds = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (256, 32, 4)))
ctx = kdev.Context(0)
for g in sorted({1, 16, G}):
    r = bench.batched_elim_rounds(ctx, lib(), errors, np.random.default_rng(3), k=k, G=g, rounds=rounds)
    print(json.dumps(r), flush=True)
r = bench.batched_elim(ctx, lib(), errors, np.random.default_rng(3), k=k, G=G)
print(json.dumps(r), flush=True)
