import ctypes, os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from kodr_amd import device
p = ctypes.CDLL(os.path.join(HERE, "libm0.so"))
ctx = device.Context(0)
out = ctx.alloc(64)
p.m0_run(ctypes.c_void_p(out), ctypes.c_void_p(ctx.stream))
ctx.synchronize()
print("M0 in index mode: after on(8) = %#x, after +8 = %#x, after off = %#x" % tuple(ctx.d2h(out, 12).view(np.uint32)))
