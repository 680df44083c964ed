"""The multi-workgroup elimination beside a kernel that holds most of the
GPU (tests/cpp/occupy.hip: every CU but a few taken by a 1024-thread
workgroup with 150 KiB of LDS for 60 ms, on another stream): gf_elim_mc2
needs all of a launch's workgroups resident, and here most cannot start.
The resident ones stop after a bounded wait (gf_elim.hip kMcPollSpins) and
the host gives up on decoders that never reported (capi.cpp kElimGiveUp), so
the batched AddPiece call returns within 10 ms -- not after the 60 ms kernel
-- and every decoder ends in kodr's state (the host route: the oracle's
literal decoder, decoder_state.go:15-182, is the reference)."""
import ctypes
import os
import time

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors
from kodr_amd._codec import elim_stats

pytestmark = pytest.mark.gpu
U8P = _lib._u8p
HERE = os.path.dirname(os.path.abspath(__file__))


def _occupier():
    lib = ctypes.CDLL(os.path.join(HERE, "cpp", "libkodr_occupy.so"))  # built by __graft_entry__.build()
    lib.kodr_test_stream_create.restype = ctypes.c_void_p
    lib.kodr_test_occupy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int]
    lib.kodr_test_stream_sync.argtypes = [ctypes.c_void_p]
    lib.kodr_test_stream_destroy.argtypes = [ctypes.c_void_p]
    return lib


def _add(lib, hs, ds, k, pitch, L):
    G = len(hs)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    rws = (ctypes.c_void_p * G)(*ds)
    counts = (ctypes.c_size_t * G)(*([k + 2] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(lib.rlnc_decoders_add_pieces_gpu(arr, G, rws, counts, pitch, L, cons, sts))
    return cons, sts


def test_elimination_beside_a_long_kernel_returns_early(gpu_ctx):
    lib = _lib.lib()
    occ = _occupier()
    k, L, G = 256, 256, 16
    rng = np.random.default_rng(99)
    hs, ds, Ps, Vs, Cs = [], [], [], [], []
    pitch = (k + L + 15) // 16 * 16
    for g in range(G):
        V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        C = oracle.encode(P, V)
        rows = np.zeros((k + 2, pitch), np.uint8)
        rows[:, :k] = V
        rows[:, k:k + L] = C
        d = gpu_ctx.alloc(rows.nbytes)
        gpu_ctx.h2d(d, rows)
        h = ctypes.c_void_p()
        errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
        hs.append(h)
        ds.append(d)
        Ps.append(P)
        Vs.append(V)
        Cs.append(C)
    gpu_ctx.synchronize()
    # one identical call first, on throwaway decoders: the context's pinned
    # status buffer and the pool's row buffers are allocated there (an
    # allocation may wait for the device, i.e. for the occupier) -- the timed
    # call below then allocates nothing
    warm = []
    for g in range(G):
        h = ctypes.c_void_p()
        errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
        warm.append(h)
    _add(lib, warm, ds, k, pitch, L)
    for h in warm:
        lib.rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    ncu = occ.kodr_test_cu_count(0)
    assert ncu > 8
    s2 = occ.kodr_test_stream_create(0)
    assert s2
    assert occ.kodr_test_occupy(s2, ncu - 4, 60.0, 150 * 1024) == 0
    time.sleep(0.003)  # the occupier's workgroups are resident
    t0 = time.perf_counter()
    cons, sts = _add(lib, hs, ds, k, pitch, L)
    dt = time.perf_counter() - t0
    routes = [elim_stats(h) for h in hs]
    occ.kodr_test_stream_sync(s2)
    gpu_ctx.synchronize()
    print(f"call {dt * 1e3:.2f} ms; routes {routes}")
    assert dt <= 0.010, (dt, routes)
    for g in range(G):
        ref = oracle.Decoder(k)
        n_ok = 0
        for i in range(k + 2):
            if ref.add(Vs[g][i], Cs[g][i]) != 0:
                break
            n_ok += 1
        assert cons[g] == n_ok and sts[g] in (0, 3)
        assert lib.rlnc_decoder_useful(hs[g]) == ref.useful()
        assert bool(lib.rlnc_decoder_is_decoded(hs[g])) == ref.is_decoded()
        out = np.empty((k, L), np.uint8)
        errors.check(lib.rlnc_decoder_get_pieces(hs[g], out.ctypes.data_as(U8P)))
        assert np.array_equal(out, Ps[g]), g
    for h in hs:
        lib.rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    for d in ds:
        gpu_ctx.free(d)
    occ.kodr_test_stream_destroy(s2)
