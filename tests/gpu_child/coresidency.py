"""Child process of tests/test_gpu_coresidency.py (test infrastructure): the
batched GPU AddPiece of 16 k = 256 decoders while a kernel holds every CU
but 4 for 60 ms, in a process with no other streams than this scenario's
(the context's own, the occupier's): streams beyond GPU_MAX_HW_QUEUES share
hardware queues, and a stream that shares one with the long kernel waits for
it whatever the library does.  Prints one JSON line: the call's wall time,
each decoder's route and whether its state and pieces match the oracle."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from kodr_amd import _lib, device, errors  # noqa: E402
from kodr_amd._codec import elim_stats  # noqa: E402

U8P = _lib._u8p


def occupier():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "cpp", "libkodr_occupy.so"))  # built by __graft_entry__.build()
    lib.kodr_test_stream_create.restype = ctypes.c_void_p
    lib.kodr_test_stream_create_high.restype = ctypes.c_void_p
    lib.kodr_test_occupy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int]
    lib.kodr_test_stream_sync.argtypes = [ctypes.c_void_p]
    lib.kodr_test_stream_destroy.argtypes = [ctypes.c_void_p]
    return lib


def add(lib, hs, ds, k, pitch, L):
    G = len(hs)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    rws = (ctypes.c_void_p * G)(*ds)
    counts = (ctypes.c_size_t * G)(*([k + 2] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(lib.rlnc_decoders_add_pieces_gpu(arr, G, rws, counts, pitch, L, cons, sts))
    return cons, sts


def run(own_priority=False):
    """own_priority: the scenario's context runs on a stream of the device's
    highest priority, created here (the condition INTEGRATION.md states: a
    context's stream must not share a hardware queue with a foreign
    long-running kernel)."""
    lib = _lib.lib()
    occ = occupier()
    hs_stream = occ.kodr_test_stream_create_high(0) if own_priority else None
    if own_priority:
        assert hs_stream
    ctx = device.Context(0, stream=hs_stream)
    k, L, G = 256, 256, 16
    rng = np.random.default_rng(99)
    pitch = (k + L + 15) // 16 * 16
    hs, ds, Ps, Vs, Cs = [], [], [], [], []
    for g in range(G):
        V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        C = oracle.encode(P, V)
        rows = np.zeros((k + 2, pitch), np.uint8)
        rows[:, :k] = V
        rows[:, k:k + L] = C
        d = ctx.alloc(rows.nbytes)
        ctx.h2d(d, rows)
        h = ctypes.c_void_p()
        errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
        hs.append(h)
        ds.append(d)
        Ps.append(P)
        Vs.append(V)
        Cs.append(C)
    ctx.synchronize()
    # one identical call first, on throwaway decoders: the context's pinned
    # buffers, streams and the pool's row buffers are allocated there (an
    # allocation may wait for the device, i.e. for the occupier)
    warm = []
    for g in range(G):
        h = ctypes.c_void_p()
        errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
        warm.append(h)
    add(lib, warm, ds, k, pitch, L)
    for h in warm:
        lib.rlnc_decoder_destroy(h)
    ctx.synchronize()
    ncu = occ.kodr_test_cu_count(0)
    assert ncu > 8
    s2 = occ.kodr_test_stream_create(0)
    assert s2
    assert occ.kodr_test_occupy(s2, ncu - 4, 60.0, 150 * 1024) == 0
    time.sleep(0.003)  # the occupier's workgroups are resident
    t0 = time.perf_counter()
    cons, sts = add(lib, hs, ds, k, pitch, L)
    dt = time.perf_counter() - t0
    routes = [elim_stats(h) for h in hs]
    occ.kodr_test_stream_sync(s2)
    ctx.synchronize()
    ok = []
    for g in range(G):
        ref = oracle.Decoder(k)
        n_ok = 0
        for i in range(k + 2):
            if ref.add(Vs[g][i], Cs[g][i]) != 0:
                break
            n_ok += 1
        good = cons[g] == n_ok and sts[g] in (0, 3) and lib.rlnc_decoder_useful(hs[g]) == ref.useful() and \
            bool(lib.rlnc_decoder_is_decoded(hs[g])) == ref.is_decoded()
        out = np.empty((k, L), np.uint8)
        errors.check(lib.rlnc_decoder_get_pieces(hs[g], out.ctypes.data_as(U8P)))
        ok.append(bool(good and np.array_equal(out, Ps[g])))
    for h in hs:
        lib.rlnc_decoder_destroy(h)
    ctx.synchronize()
    for d in ds:
        ctx.free(d)
    occ.kodr_test_stream_destroy(s2)
    ctx.close()
    if hs_stream:
        occ.kodr_test_stream_destroy(ctypes.c_void_p(hs_stream))
    return {"call_s": dt, "routes": routes, "ok": ok}


def main():
    print(json.dumps(run()), flush=True)


if __name__ == "__main__":
    main()
