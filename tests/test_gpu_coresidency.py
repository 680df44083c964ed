"""The multi-workgroup elimination beside a kernel that holds most of the
GPU (tests/cpp/occupy.hip: every CU but a few taken by a 1024-thread
workgroup with 150 KiB of LDS for 60 ms, on another stream): gf_elim_mc2
needs all of a launch's workgroups resident, and here most cannot start.
The resident ones stop after a bounded wait (gf_elim.hip kMcPollSpins), the
host gives up on decoders that never reported (capi_decoder.cpp kElimGiveUp) and
takes kodr's route with the coding vectors downloaded beside the launch, so
the batched AddPiece call returns within 10 ms -- not after the 60 ms kernel
-- and every decoder ends in kodr's state (the host route: the oracle's
literal decoder, decoder_state.go:15-182, is the reference).

The scenario runs twice: in a child process (tests/gpu_child/coresidency.py)
with only its own streams, and inside this pytest process after every other
GPU test has created its contexts.  Streams beyond GPU_MAX_HW_QUEUES (4 on the
box) share hardware queues; in round 5 the give-up route's vector download
ran on a normal-priority stream, landed on the occupier's queue inside the
long session and waited for it (57 ms, profiles/r05/coresidency/).  The
download stream is now of the highest priority (a hardware queue pool of its
own, capi_decoder.cpp ctx_aux_after_rows)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_elimination_beside_a_long_kernel_returns_early():
    if not os.path.exists(os.path.join(HERE, "cpp", "libkodr_occupy.so")):
        pytest.skip("test occupier not built (__graft_entry__.build)")
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_child", "coresidency.py")], capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(f"call {res['call_s'] * 1e3:.2f} ms; routes {res['routes']}")
    assert all(res["ok"]), res
    assert res["call_s"] <= 0.010, res



@pytest.mark.parametrize("hook", [False, True])
def test_work_queued_ahead_does_not_start_the_give_up_clock(hook):
    """More than kElimGiveUp (5 ms) of work queued ahead of the launch on the
    context's own stream (the occupier, one workgroup for 20 ms, standing in
    for a large encode or the previous step's GetPieces) must not count
    against the launch: the give-up clock starts when the launch becomes
    eligible (capi_decoder.cpp elim_direct_wait, `ready`).  Every decoder
    stays on the GPU route and equals the oracle.  hook: through
    rlnc_decoders_add_pieces_gpu_hook, whose hook must run only once that
    work is done (the launch is next on the device), not right after the
    launch is queued."""
    if not os.path.exists(os.path.join(HERE, "cpp", "libkodr_occupy.so")):
        pytest.skip("test occupier not built (__graft_entry__.build)")
    import ctypes
    import time

    import numpy as np

    import oracle
    from kodr_amd import _lib, device, errors
    from kodr_amd._codec import elim_stats
    spec_path = os.path.join(HERE, "gpu_child", "coresidency.py")
    import importlib.util
    spec = importlib.util.spec_from_file_location("kodr_coresidency_child", spec_path)
    child = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(child)
    lib = _lib.lib()
    occ = child.occupier()
    ctx = device.Context(0)
    try:
        k, L, G = 256, 256, 8
        rng = np.random.default_rng(1234)
        pitch = (k + L + 15) // 16 * 16
        hs, ds, Ps, Vs, Cs = [], [], [], [], []
        for g in range(G):
            V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
            P = rng.integers(0, 256, (k, L), dtype=np.uint8)
            C = oracle.encode(P, V)
            rows = np.zeros((k + 2, pitch), np.uint8)
            rows[:, :k], rows[:, k:k + L] = V, C
            d = ctx.alloc(rows.nbytes)
            ctx.h2d(d, rows)
            h = ctypes.c_void_p()
            errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
            hs.append(h)
            ds.append(d)
            Ps.append(P)
            Vs.append(V)
            Cs.append(C)
        # warm call on throwaway decoders (pinned buffers, streams, pool blocks)
        warm = []
        for g in range(G):
            h = ctypes.c_void_p()
            errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
            warm.append(h)
        child.add(lib, warm, ds, k, pitch, L)
        for h in warm:
            lib.rlnc_decoder_destroy(h)
        ctx.synchronize()
        assert occ.kodr_test_occupy(ctypes.c_void_p(ctx.stream), 1, 20.0, 1024) == 0
        t0 = time.perf_counter()
        t_hook = []
        if hook:
            arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
            rws = (ctypes.c_void_p * G)(*ds)
            counts = (ctypes.c_size_t * G)(*([k + 2] * G))
            cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()

            def _hook(_u):
                t_hook.append(time.perf_counter())
                return None
            fn = _lib.HOOK_FN(_hook)
            errors.check(lib.rlnc_decoders_add_pieces_gpu_hook(arr, G, rws, counts, pitch, L, cons, sts, fn, None))
        else:
            cons, sts = child.add(lib, hs, ds, k, pitch, L)
        dt = time.perf_counter() - t0
        if hook:
            assert len(t_hook) == 1
            assert t_hook[0] - t0 >= 0.015, t_hook[0] - t0  # called once the occupier was done
        routes = [elim_stats(h) for h in hs]
        print(f"call {dt * 1e3:.2f} ms; routes {routes}")
        assert dt >= 0.015, dt  # it did wait for the queued work
        assert all(r["gpu"] == 1 and r["host_after_gpu"] == 0 for r in routes), routes
        for g in range(G):
            assert cons[g] == k and sts[g] in (0, 3)  # (3: the rows past k, kodr's ErrAllUsefulPiecesReceived)
            out = np.empty((k, L), np.uint8)
            errors.check(lib.rlnc_decoder_get_pieces(hs[g], out.ctypes.data_as(_lib._u8p)))
            assert np.array_equal(out, Ps[g])
        for h in hs:
            lib.rlnc_decoder_destroy(h)
        ctx.synchronize()
        for d in ds:
            ctx.free(d)
    finally:
        ctx.close()
