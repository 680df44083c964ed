"""Config-5 relay phases on one GPU (world size 1: the ring shift is a device
copy): encode k wire rows with device vectors, shift, recoder create from the
device rows, recode k pieces.  Times each phase (ms, best of reps)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes
import numpy as np
import torch
import torch.distributed as dist
import bench
from kodr_amd import dist as kdist, errors
from kodr_amd import device as kdev
from kodr_amd._lib import lib

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("gloo", rank=0, world_size=1)
L_ = lib()
ctx = kdev.Context(0)
k, L = 256, 131072
rng = np.random.default_rng(3)
data = rng.integers(0, 256, k * L, dtype=np.uint8)
h = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 0, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                    ctypes.byref(h)))
print(bench.run_relay(ctx, L_, errors, h, k, L, rng, torch, dist, kdist), flush=True)
L_.rlnc_encoder_destroy(h)
dist.destroy_process_group()
