"""rlnc_decoders_add_pieces_gpu_hook (include/kodr_rlnc.h): the caller's hook
runs exactly once per call -- after the first elimination launch, or on the
way out when no batch goes to the GPU -- and the decoders end exactly as
through rlnc_decoders_add_pieces_gpu (kodr's state: full/decoder.go:50-66,
decoder_state.go:15-182), checked against the oracle's literal decoder's
decoded pieces; a hook that returns an event orders the call's row copies
behind the caller's work."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, device, errors

pytestmark = pytest.mark.gpu


def _rows(rng, V, P, k, L, pitch):
    rows = np.zeros((V.shape[0], pitch), np.uint8)
    rows[:, :k], rows[:, k:k + L] = V, oracle.encode(P, V)
    return rows


def _run(gpu_ctx, G, k, L, systematic=False, hook_event=False, seed=5):
    lib = _lib.lib()
    rng = np.random.default_rng(seed)
    n, pitch = k + 2, (k + L + 15) // 16 * 16
    Ps, ds, hs = [], [], []
    for g in range(G):
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        if systematic:  # the first k pieces uncoded (systematic/encoder.go:82-109), then two coded
            V = np.vstack([np.eye(k, dtype=np.uint8), rng.integers(0, 256, (2, k), dtype=np.uint8)])
        else:
            V = rng.integers(0, 256, (n, k), dtype=np.uint8)
        d = gpu_ctx.alloc(n * pitch)
        gpu_ctx.h2d(d, _rows(rng, V, P, k, L, pitch))
        h = ctypes.c_void_p()
        errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
        Ps.append(P)
        ds.append(d)
        hs.append(h)
    calls = []
    other = device.Context(0) if hook_event else None  # the caller's work on a context of its own
    ev = other.event() if hook_event else None

    def _hook(_u):
        calls.append(1)
        if ev is not None:
            other.record(ev)
            return ev.value
        return None
    fn = _lib.HOOK_FN(_hook)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    rws = (ctypes.c_void_p * G)(*ds)
    counts = (ctypes.c_size_t * G)(*([n] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(lib.rlnc_decoders_add_pieces_gpu_hook(arr, G, rws, counts, pitch, L, cons, sts, fn, None))
    assert len(calls) == 1, calls
    for g in range(G):
        assert cons[g] == k and sts[g] in (0, 3), (g, cons[g], sts[g])  # 3: kodr's ErrAllUsefulPiecesReceived
        out = np.empty((k, L), np.uint8)
        errors.check(lib.rlnc_decoder_get_pieces(hs[g], out.ctypes.data_as(_lib._u8p)))
        assert np.array_equal(out, Ps[g]), g
    for h in hs:
        lib.rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    for d in ds:
        gpu_ctx.free(d)
    if other is not None:
        other.synchronize()
        lib.rlnc_event_destroy(ev)
        other.close()


@pytest.mark.parametrize("G,k,L", [(4, 256, 4096), (16, 256, 1024), (3, 64, 2048)])
def test_hook_once_gpu_batches(gpu_ctx, G, k, L):
    _run(gpu_ctx, G, k, L)


def test_hook_once_when_the_host_takes_the_batch(gpu_ctx):
    # systematic-looking batches are solved on the host (no elimination
    # launch): the hook still runs once, on the way out
    _run(gpu_ctx, 4, 256, 2048, systematic=True)


def test_hook_event_orders_the_row_copies(gpu_ctx):
    _run(gpu_ctx, 8, 256, 4096, hook_event=True)
