import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kodr_amd import device
p = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvalu.so"))
ctx = device.Context(0)
out = ctx.alloc(64 << 20)
st = ctypes.c_void_p(ctx.stream)
e0, e1 = ctx.event(), ctx.event()
names = {0: "perm(sel=a&7)+and", 1: "perm(a,t,sel)", 2: "bitop3", 3: "xor+add", 4: "perm(t0,t1,a)"}
iters = 2000
for op in range(5):
    for blocks in (2048, 8192):
        p.probe_valu(op, ctypes.c_void_p(out), blocks, 10, st)
        ctx.record(e0)
        p.probe_valu(op, ctypes.c_void_p(out), blocks, iters, st)
        ctx.record(e1)
        ms = device.Context.elapsed_ms(e0, e1)
        insts = blocks * 4 * iters * 16 * 8  # wave-instructions of the op
        lane_ops = insts * 64
        print(f"{names[op]:18s} blocks={blocks:5d} {ms:8.3f} ms  {lane_ops/ms/1e9:8.2f} T lane-op/s  "
              f"cycles/wave-inst/SIMD @2.4GHz = {ms*1e-3*2.4e9*1024/insts:.2f}", flush=True)
