#!/usr/bin/env python3
"""Headline benchmark: Full-RLNC encode of a 32 MiB generation split into 256
pieces (BASELINE.json configs[1]) on MI355X, device-resident, coded MB/s.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--gens G]

One step = one pass of the hot path: B coded pieces of one resident generation
(one kernel launch: B coding vectors x the k x L generation; gf_bs_kernel
for B >= 9, gf_gemm_kernel below).  The G
generations rotate so that consecutive steps stream from HBM, not from the
256 MiB Infinity Cache.  Metric accounting is kodr's own: each coded piece is
worth SetBytes = S + padding + (k + L) bytes (benches/full/encoder_test.go:53),
reported in 10^6 B/s like Go's MB/s.

Multi-GPU (torchrun, one process per GPU): generations are independent, so
every rank encodes its own G generations with no data-path collective (weak
scaling); value = all ranks' coded bytes / max-over-ranks time.

The JSON line also carries the roofline of the dominant kernel (gf_bs_kernel,
timed with HIP events on the stream it runs on) and a CPU baseline: the
kodr-equivalent scalar restatement (oracle/, one core) timed on a bounded
sample of the same workload on this host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K_PIECES, L_BYTES = 256, 131072          # 32 MiB / 256 pieces
HBM_PEAK_GBS = 8000.0                     # MI355X_MICROARCH.md: 8.0 TB/s spec


class host_elimination:
    """The comparisons' host legs run kodr's elimination on the host:
    rlnc_decoder_add_pieces and the lazy AddPiece flush would otherwise take
    the GPU elimination themselves for large full batches (capi_decoder.cpp
    dec_route_gpu, the context's rlnc_ctx_set_route_min_k)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def __enter__(self):
        self.prev = self.ctx.route_min_k
        self.ctx.set_route_min_k(100000)

    def __exit__(self, *exc):
        self.ctx.set_route_min_k(self.prev)


def setbytes(k, L, padding=0):
    # benches/full/encoder_test.go:53  SetBytes(total + padding + CodedPieceLen)
    return k * L + padding + (k + L)


def cpu_baseline(seconds=10.0):
    """Time oracle/ (kodr-equivalent scalar Go restatement, 1 thread) encoding
    32 MiB/256 coded pieces for ~`seconds`."""
    import numpy as np
    import oracle
    rng = np.random.default_rng(1)
    P = rng.integers(0, 256, (K_PIECES, L_BYTES), dtype=np.uint8)
    V = rng.integers(0, 256, (64, K_PIECES), dtype=np.uint8)
    # kodr is single-threaded: pin this process to one core for the sample,
    # as `taskset -c <core>` would (CPU-baseline plan)
    prev = os.sched_getaffinity(0)
    core = min(prev)
    os.sched_setaffinity(0, {core})
    try:
        oracle.encode(P, V[:1])  # warm tables / pages
        n, t0 = 0, time.perf_counter()
        while True:
            oracle.encode(P, V[n % 64:n % 64 + 1])
            n += 1
            dt = time.perf_counter() - t0
            if dt >= seconds and n >= 3:
                break
    finally:
        os.sched_setaffinity(0, prev)
    return {"value": round(n * setbytes(K_PIECES, L_BYTES) / dt / 1e6, 2), "unit": "MB/s",
            "cores": 1, "kind": "port",
            "sample": f"{n} coded pieces of 32MiB/256 by oracle/kodr_oracle.c (scalar restatement of "
                      f"data.go:19-29 + gf256.go:109-118), {dt:.1f}s pinned to core {core} of "
                      f"{os.cpu_count()} ({_cpu_model()})"}


def cpu_baseline_decode(seconds=6.0, k=K_PIECES, L=L_BYTES, widths=(256, 1024)):
    """kodr's decode of k + 2 coded pieces by oracle/ (decoder_state.go's
    literal loops, full/decoder.go's AddPiece; one core) on column slices of a
    32 MiB/256 generation.  Decode is column-separable (decoder_state.go:66-73,
    105-112, 130-132: the data bytes of a column meet only that column), so a
    slice of w columns does the whole coefficient side and w/L of the data
    side: t(w) = a + b w, fitted at two widths (best of the repetitions that
    fit in `seconds`), is evaluated at w = L."""
    import numpy as np
    import oracle
    rng = np.random.default_rng(2)
    n = k + 2
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    prev = os.sched_getaffinity(0)
    core = min(prev)
    os.sched_setaffinity(0, {core})
    best = {}
    try:
        for w in widths:
            P = rng.integers(0, 256, (k, w), dtype=np.uint8)
            C = oracle.encode(P, V)
            t_end, reps = time.perf_counter() + seconds / len(widths), 0
            while reps < 2 or time.perf_counter() < t_end:
                t0 = time.perf_counter()
                d = oracle.Decoder(k)
                for i in range(n):
                    if d.add(V[i], C[i]) == 3:
                        break
                dt = time.perf_counter() - t0
                assert d.is_decoded() and np.array_equal(np.stack([d.get_piece(i)[1] for i in range(k)]), P)
                best[w] = min(best.get(w, dt), dt)
                reps += 1
    finally:
        os.sched_setaffinity(0, prev)
    (w1, w2) = widths
    b = (best[w2] - best[w1]) / (w2 - w1)
    a = best[w1] - b * w1
    t_full = a + b * L
    return {"decode_s": round(t_full, 4), "decode_MBps_decodable_len": round(k * (k + L) / t_full / 1e6, 3),
            "coefficient_side_s": round(max(a, 0.0), 5), "per_column_s": float(f"{b:.4g}"),
            "slice_s": {str(w): round(best[w], 5) for w in widths}, "cores": 1, "kind": "port",
            "sample": f"oracle.Decoder (literal decoder_state.go) fed k + 2 = {n} coded pieces of 32MiB/256 "
                      f"column slices of {widths[0]} and {widths[1]} bytes, best of the repetitions in "
                      f"{seconds:.0f}s, pinned to core {core}; t(L) = a + b L extrapolated to L = {L} "
                      f"(kodr publishes 13.07 s for this decode on an i7-1260P, README.md:142)"}


def cpu_baseline_roundtrip(enc, dec, k=K_PIECES, L=L_BYTES):
    """The encode+decode round trip of one generation on one core, from the
    two samples: k + 2 coded pieces at the encode rate, then the decode;
    kodr units as encode_decode.value."""
    n = k + 2
    t_enc = n * setbytes(k, L) / (enc["value"] * 1e6)
    t = t_enc + dec["decode_s"]
    units = n * setbytes(k, L) + k * (k + L)
    return {"value": round(units / t / 1e6, 2), "unit": "MB/s", "cores": 1, "kind": "port",
            "roundtrip_s_per_generation": round(t, 4), "encode_s": round(t_enc, 4), "decode_s": dec["decode_s"],
            "sample": "k + 2 coded pieces at cpu_baseline's oracle encode rate + cpu_baseline_decode's extrapolated "
                      "oracle decode, one core; kodr units as encode_decode.value ((k+2) x SetBytes + DecodableLen "
                      "per generation)", "decode_detail": dec}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def c1_roundtrip(ctx, L_, errors, rng):
    """BASELINE config 1 (1 MiB / 16 pieces): kodr's own CPU round trip
    (benches/full: encode k+2 coded pieces, decode) by the oracle on one core,
    and the same round trip through the engine's host API."""
    import ctypes
    import numpy as np
    import oracle
    k, L = 16, 65536
    u8p = ctypes.POINTER(ctypes.c_uint8)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
    t0 = time.perf_counter()
    C = oracle.encode(P, V)
    d = oracle.Decoder(k)
    for i in range(k + 2):
        if d.add(V[i], C[i]) == 3:
            break
    dec = np.stack([d.get_piece(i)[1] for i in range(k)])
    t_cpu = time.perf_counter() - t0
    wire = np.empty((k + 2, k + L), np.uint8)
    outp = np.empty((k, L), np.uint8)
    best = None
    for rep in range(3):
        t0 = time.perf_counter()
        eh, dh = ctypes.c_void_p(), ctypes.c_void_p()
        errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(u8p), k, L, ctypes.byref(eh)))
        errors.check(L_.rlnc_encoder_coded_pieces(eh, V.ctypes.data_as(u8p), k + 2, wire.ctypes.data_as(u8p)))
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
        consumed = ctypes.c_size_t()
        st = L_.rlnc_decoder_add_pieces(dh, wire.ctypes.data_as(u8p), k + 2, k + L, L, 0, ctypes.byref(consumed))
        if st != 3:
            errors.check(st)
        errors.check(L_.rlnc_decoder_get_pieces(dh, outp.ctypes.data_as(u8p)))
        t = time.perf_counter() - t0
        L_.rlnc_decoder_destroy(dh)
        L_.rlnc_encoder_destroy(eh)
        best = t if best is None else min(best, t)
    return {"cpu_oracle_s": round(t_cpu, 6), "gpu_host_api_s": round(best, 6),
            "roundtrip_ok": bool(np.array_equal(dec, P) and np.array_equal(outp, P)),
            "note": "encode k+2 pieces + decode, host buffers in and out; kodr publishes only the "
                    "encode rate for this shape (README.md:73)"}


class HeadlineStep:
    """The timed step, shared with tests/test_gpu_headline.py (which runs it
    once and compares every piece with the oracle, and pins its launch plan).

    G resident generations of k x L (seeded random bytes) are uploaded and
    prepared (rlnc_encoder_prepare: the bit-sliced twin) at construction,
    outside the timed loop, as kodr's bench constructs its encoder before
    b.Loop (benches/full/encoder_test.go:47-56); the cost is reported apart
    (construct_ms_per_generation).  A step: B coded pieces of every resident
    generation (full/encoder.go:61-71 B times per generation, vectors drawn
    per piece) as ONE grouped launch (rlnc_encoder_group_coded_pieces_device:
    the launch and the kernel's ramp and tail are paid once per G
    generations, each generation read once); per_generation=True: one
    launch per generation, rotating over the G.  Vectors rotate over nvec
    pre-drawn sets (host copy in self.V)."""

    def __init__(self, ctx, L_, errors, k, L, B, G, grouped=True, rng=None, nvec=None, keep_data=False):
        import ctypes
        import numpy as np
        self.ctx, self.L_, self.errors = ctx, L_, errors
        self.k, self.L, self.B, self.G, self.grouped = k, L, B, G, grouped
        rng = rng if rng is not None else np.random.default_rng(0x6B6F6472)
        datas = [rng.integers(0, 256, k * L, dtype=np.uint8) for _ in range(G)]
        self.encs = []
        ctx.synchronize()
        tc0 = time.perf_counter()
        for g in range(G):
            h = ctypes.c_void_p()
            errors.check(L_.rlnc_encoder_create(ctx.handle, 0, datas[g].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                                k, L, ctypes.byref(h)))
            errors.check(L_.rlnc_encoder_prepare(h))
            self.encs.append(h)
        ctx.synchronize()
        self.construct_ms = (time.perf_counter() - tc0) * 1e3 / G
        self.datas = datas if keep_data else None
        self.per_step = G if grouped else 1            # generations per step
        self.nvec = nvec or (8 if grouped else 64)
        self.V = rng.integers(0, 256, (self.nvec, self.per_step, B, k), dtype=np.uint8)
        self.dV = ctx.alloc(self.V.nbytes)
        ctx.h2d(self.dV, self.V)
        self.dOut = ctx.alloc(self.per_step * B * L)
        self.enc_arr = (ctypes.c_void_p * G)(*[e.value for e in self.encs])

    def step(self, i):
        k, L, B = self.k, self.L, self.B
        dv = self.dV + (i % self.nvec) * self.per_step * B * k
        if self.grouped:
            self.errors.check(self.L_.rlnc_encoder_group_coded_pieces_device(self.enc_arr, self.G, dv, B, self.dOut, L))
        else:
            self.errors.check(self.L_.rlnc_encoder_coded_pieces_device(self.encs[i % self.G], dv, B, self.dOut, L))

    def close(self):
        for h in self.encs:
            self.L_.rlnc_encoder_destroy(h)
        self.encs = []
        self.ctx.free(self.dV)
        self.ctx.free(self.dOut)


class RoundTripStep:
    """The metric's encode+decode (configs[1] encode + configs[2] decode) as a
    timed step over the G resident generations, shared with
    tests/test_gpu_headline.py (which runs it and compares every decoded
    byte).  Coding vectors: nsets sets of n = k + 2 per generation drawn on
    the host up front (kodr draws them per piece from crypto/rand,
    data.go:90-95; fresh sets rotate between steps) and written into the
    vector columns of nsets wire-row buffers (CodedPiece.Flatten layout,
    data.go:52-57, pitch round_up(k + L, 256)).  A step:
      1. ONE grouped encode launch (rlnc_encoder_group_coded_pieces_device,
         gf_bs_kernel) writes the n coded pieces of every generation into
         the piece columns of set i % nsets -- full/encoder.go:61-71 n times
         per generation; HIP events around it;
      2. G fresh decoders take their n wire rows in ONE batched AddPiece call
         (rlnc_decoders_add_pieces_gpu: the multi-workgroup elimination,
         gf_elim_mc_kernel, then the rows' bit-sliced twin) --
         full/decoder.go:50-66 row by row, same state;
      3. ONE grouped GetPieces (rlnc_decoders_get_pieces_device) writes the
         G decoded generations to device memory; HIP events around it;
      4. the next step's G decoders are constructed while GetPieces runs
         (host only), then this step's decoders are destroyed (their buffers
         go back to the pool ordered on the stream, no host wait).
    Pipelined (dctx: the decoders' own context, so their own stream): the
    encoders stay on ctx, and once step i's AddPiece call has returned (its
    elimination done), step i + 1's encode -- which depends on nothing of
    step i's decode -- is queued on the encoders' stream before step i's
    GetPieces, so it runs beside step i's twin copy and GetPieces instead of
    after them.  The decoders' stream waits for the encode it reads (an
    event); the encode of step i + 1 rewrites the wire rows of set
    (i + 1) % nsets, which only step i - 1's twin copy read, and that copy
    precedes step i's elimination on the decoders' stream (done when the
    AddPiece call returns; a given-up decoder's give-up clock starts only
    once everything ahead of the launch is done).  Within the timed phase
    no encode is queued past its last step (begin_phase), so K timed steps
    are exactly K encodes and K decodes.
    Decoder construction stays inside the timed steps (each step constructs
    the next one's; the first warmup step its own); kodr's decoder bench
    builds its decoder outside the timer (benches/full/decoder_test.go:71-94)."""

    def __init__(self, ctx, L_, errors, encs, k, L, rng, nsets=2, dctx=None, overlap="elim"):
        import ctypes
        import numpy as np
        self.ctx, self.L_, self.errors, self.encs = ctx, L_, errors, encs
        self.dctx = dctx if dctx is not None else ctx
        self.pipelined = self.dctx is not ctx
        # what step i + 1's encode runs beside: "elim" -- step i's elimination
        # (queued from inside the AddPiece call right after its launch) and
        # twin copy; "copy" -- the twin copy only (queued after the call); both
        # make GetPieces wait for it; "get" -- the copy and GetPieces
        self.overlap = overlap
        self.k, self.L, self.G, self.n = k, L, len(encs), k + 2
        self.W = (k + L + 255) // 256 * 256
        G, n, W = self.G, self.n, self.W
        self.V = rng.integers(0, 256, (nsets, G, n, k), dtype=np.uint8)
        self.dV, self.dW = [], []
        wire = np.zeros((G * n, W), np.uint8)
        for s_ in range(nsets):
            dv, dw = ctx.alloc(G * n * k), ctx.alloc(G * n * W)
            ctx.h2d(dv, self.V[s_])
            wire[:, :k] = self.V[s_].reshape(G * n, k)
            ctx.h2d(dw, wire)
            self.dV.append(dv)
            self.dW.append(dw)
        del wire
        self.dO = ctx.alloc(G * k * L)
        self.earr = (ctypes.c_void_p * G)(*[e.value for e in encs])
        self.rows = [(ctypes.c_void_p * G)(*[dw + g * n * W for g in range(G)]) for dw in self.dW]
        self.counts = (ctypes.c_size_t * G)(*([n] * G))
        self.ev = [[ctx.event() for _ in range(4)] for _ in range(2)]  # untimed steps (by parity)
        self.pend = []                                 # timed steps' events, read after the steps
        self.spare = []
        self._t_enc, self.t_add, self._t_get, self._t_gpu_add, self.ok = [], [], [], [], True
        self.next_decs = None
        self.plans = None
        self.ahead = None      # (step, events) of the encode a pipelined step queued for the next one
        self.limit = None      # no encode is queued for a step >= limit (None: no limit)
        self.encodes = 0       # encode launches so far, and at the start of the current phase
        self.encodes_before_phase = 0

    def begin_phase(self, limit=None):
        """A new phase of steps 0, 1, ... (limit: its length, when known): an
        encode queued ahead by the previous phase is dropped (its result is
        never read; the barrier between the phases waits for it)."""
        self.ahead, self.limit = None, limit
        self.encodes_before_phase = self.encodes

    def synchronize(self):
        self.ctx.synchronize()
        if self.pipelined:
            self.dctx.synchronize()

    def _decoders(self):
        import ctypes
        decs = []
        for g in range(self.G):
            h = ctypes.c_void_p()
            self.errors.check(self.L_.rlnc_decoder_create(self.dctx.handle, self.k, ctypes.byref(h)))
            decs.append(h)
        return decs

    def _events(self, i, timed):
        if not timed:
            return self.ev[i & 1]
        return self.spare.pop() if self.spare else [self.ctx.event() for _ in range(4)]

    def _encode(self, i, e):
        s_ = i % len(self.dW)
        self.ctx.record(e[0])
        self.errors.check(self.L_.rlnc_encoder_group_coded_pieces_device(self.earr, self.G, self.dV[s_], self.n,
                                                                         self.dW[s_] + self.k, self.W))
        self.ctx.record(e[1])
        self.encodes += 1
        if self.plans is None:   # the launches' kernel instances (first warmup step: tools/prof_roundtrip.py)
            from kodr_amd._lib import last_launch_plan
            self.plans = {"encode": last_launch_plan()}

    def step(self, i, timed=True):
        import ctypes
        L_, errors, G, k, L = self.L_, self.errors, self.G, self.k, self.L
        s_ = i % len(self.dW)
        decs = self.next_decs if self.next_decs is not None else self._decoders()
        self.next_decs = None
        darr = (ctypes.c_void_p * G)(*[x.value for x in decs])
        if self.ahead is not None and self.ahead[0] == i:
            e = self.ahead[1]                  # queued by the previous step
            self.ahead = None
        else:
            e = self._events(i, timed)
            self._encode(i, e)
        if self.pipelined:
            self.dctx.wait(e[1])              # the decoders' stream reads the rows this encode wrote
        ahead = self.pipelined and (self.limit is None or i + 1 < self.limit)
        if self.pipelined and self.overlap == "elim_sync":
            # the elimination needs all of its workgroups resident at once: an
            # encode dispatched ahead of them takes the CUs first (measured,
            # 16 x 8 workgroups then took 1.45 ms instead of 0.16).  The
            # library calls the hook only once the work ahead of the launch on
            # the decoders' stream (the previous GetPieces) is done; this
            # variant also starts the call on an idle GPU (one host wait per
            # step: the gap between GetPieces and the next elimination)
            self.dctx.synchronize()
            self.ctx.synchronize()
        ta0 = time.perf_counter()
        cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
        if ahead and self.overlap in ("elim", "elim_sync", "elim_only"):
            # step i + 1's encode queued from inside the AddPiece call, right
            # after the elimination's launch: it runs beside the elimination
            # (on the CUs its workgroups leave free) and the twin copy
            # ("elim_only": the copy waits for the encode -- the hook returns
            # its end event)
            en = self._events(i + 1, timed)

            def _hook(_u, en=en):
                self._encode(i + 1, en)
                return en[1].value if self.overlap == "elim_only" else None
            hook = _lib_hook(_hook)
            errors.check(L_.rlnc_decoders_add_pieces_gpu_hook(darr, G, self.rows[s_], self.counts, self.W, L, cons,
                                                              sts, hook, None))
        else:
            errors.check(L_.rlnc_decoders_add_pieces_gpu(darr, G, self.rows[s_], self.counts, self.W, L, cons, sts))
        ta1 = time.perf_counter()
        self.dctx.record(e[2])
        if ahead:
            if self.overlap not in ("elim", "elim_sync", "elim_only"):
                en = self._events(i + 1, timed)
                self._encode(i + 1, en)        # beside this step's twin copy (and GetPieces)
            self.ahead = (i + 1, en)
            if self.overlap in ("copy", "elim", "elim_sync", "elim_only"):
                self.dctx.wait(en[1])          # GetPieces after it: two bit-sliced launches side by side lose
        errors.check(L_.rlnc_decoders_get_pieces_device(darr, G, self.dO, L))
        self.dctx.record(e[3])
        if "get" not in self.plans:
            from kodr_amd._lib import last_launch_plan
            self.plans["get"] = last_launch_plan()
        self.ok = self.ok and all(st in (0, 3) for st in sts) and all(c == k for c in cons)
        self.next_decs = self._decoders()    # the next step's, on the host while GetPieces runs
        for x in decs:
            L_.rlnc_decoder_destroy(x)        # no host wait: the buffers go back ordered on the stream
        if timed:
            self.pend.append(e)               # (read after the timed steps: no wait inside them)
            self.t_add.append(ta1 - ta0)

    def _collect(self):
        from kodr_amd import device as kdev
        for e in self.pend:
            self._t_enc.append(kdev.Context.elapsed_ms(e[0], e[1]) / 1e3)
            self._t_gpu_add.append(kdev.Context.elapsed_ms(e[1], e[2]) / 1e3)
            self._t_get.append(kdev.Context.elapsed_ms(e[2], e[3]) / 1e3)
            self.spare.append(e)
        self.pend = []

    @property
    def t_enc(self):
        self._collect()
        return self._t_enc

    @property
    def t_get(self):
        self._collect()
        return self._t_get

    @property
    def t_gpu_add(self):
        self._collect()
        return self._t_gpu_add

    def decoded_ok(self, gens=None):
        """The last step's decoded generations against the resident ones."""
        import ctypes
        import numpy as np
        self.synchronize()
        ok = self.ok
        pitch = ctypes.c_size_t()
        for g in (gens if gens is not None else sorted({0, self.G - 1})):
            dp = self.L_.rlnc_encoder_device_pieces(self.encs[g], ctypes.byref(pitch))
            a = self.ctx.d2h(self.dO + g * self.k * self.L, self.k * self.L)
            b = self.ctx.d2h(dp, self.k * pitch.value).reshape(self.k, pitch.value)[:, :self.L].reshape(-1)
            ok = ok and bool(np.array_equal(a, b))
        return ok

    def units(self):
        """kodr units per step: (k + 2) x SetBytes (encoder bench,
        benches/full/encoder_test.go:53) + DecodableLen k (k + L) (the decoded
        generation) per generation."""
        return self.G * (self.n * setbytes(self.k, self.L) + self.k * (self.k + self.L))

    def close(self):
        self.synchronize()
        for x in self.next_decs or []:
            self.L_.rlnc_decoder_destroy(x)
        self.next_decs = None
        self.dctx.synchronize()
        for p_ in self.dV + self.dW + [self.dO]:
            self.ctx.free(p_)


def _lib_hook(fn):
    from kodr_amd._lib import HOOK_FN
    return HOOK_FN(fn)


def run_timed(step, steps, warmup, barrier, warm_s, max_warm=20000, phase=None):
    """W untimed steps, never fewer than one and never less than warm_s of
    back-to-back work (the clock transient, DESIGN.md Roofline), a barrier,
    then exactly `steps` timed steps bracketed by barriers.  phase(limit), if
    given, is called before each phase (RoundTripStep.begin_phase).  Returns
    (wall seconds of the timed steps on this rank, warmup steps run)."""
    n_warm = 0
    if phase:
        phase(None)
    tw0 = time.perf_counter()
    while n_warm < max(warmup, 1) or (time.perf_counter() - tw0 < warm_s and n_warm < max_warm):
        step(n_warm, False)
        n_warm += 1
    barrier()
    if phase:
        phase(steps)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i, True)
    barrier()
    return time.perf_counter() - t0, n_warm


def roundtrip_block(t_local, steps, warmup, n_warm, units_per_step, world, kdist, device=None):
    """The encode_decode block: whole-job kodr units over the slowest rank's
    time for `steps` round trips (aggregate, weak scaling: every rank decodes
    its own generations)."""
    t_max = kdist.max_over_ranks(t_local, device=device)
    return {"value": round(kdist.aggregate_rate(steps, units_per_step, t_max, world), 1), "unit": "MB/s",
            "n_gpus": world, "steps": steps, "warmup": warmup, "warmup_steps_run": n_warm,
            "ms_per_step": round(t_max / steps * 1e3, 5), "higher_is_better": True, "scaling": "weak",
            "units_per_step_per_rank": units_per_step}


def roundtrip_kernels(rt, k, L):
    """Per-leg figures of the timed round trips (HIP events on the context
    stream around the encode launch and the GetPieces call; the AddPiece call's
    host wall time, which ends with the transforms read back), each against
    its bound."""
    import statistics
    G, n = rt.G, rt.n
    te, ta, tg, tga = (statistics.mean(x) for x in (rt.t_enc, rt.t_add, rt.t_get, rt.t_gpu_add))
    enc_macs, get_macs, elim_macs = G * n * k * L, G * k * k * L, G * k ** 3
    return {
        "encode_launch": {"kernel": "gf_bs_kernel (grouped, B = k + 2 per generation)", "avg_us": round(te * 1e6, 2),
                          "us_per_generation": round(te / G * 1e6, 2),
                          "gf_macs_per_s": float(f"{enc_macs / te:.4g}"),
                          "issue_frac": round(enc_macs / te / VALU_FLOOR_MACS_PER_S, 4),
                          "hbm_bytes": G * (k * L + n * k + n * L),
                          "hbm_frac": round(G * (k * L + n * k + n * L) / te / 1e9 / HBM_PEAK_GBS, 4),
                          "plan": rt.plans["encode"]},
        "add_pieces_call": {"avg_us": round(tga * 1e6, 2), "us_per_generation": round(tga / G * 1e6, 2),
                            "call_wall_us": round(ta * 1e6, 2),
                            "elimination_gf_macs": elim_macs,
                            "row_bytes": G * 2 * n * L,
                            "note": "avg_us: the context stream from the encode's end to GetPieces' start (HIP "
                                    "events): the elimination (gf_elim_mc_kernel), then the rows' bit-sliced twin "
                                    "(read n L, write n L per generation: compact rows, no plain copy); "
                                    "call_wall_us: the call's host wall time, which also waits for the work queued "
                                    "ahead of its launch"},
        "get_pieces_call": {"kernel": "gf_bs_kernel (grouped T x R)", "avg_us": round(tg * 1e6, 2),
                            "us_per_generation": round(tg / G * 1e6, 2),
                            "gf_macs_per_s": float(f"{get_macs / tg:.4g}"),
                            "issue_frac": round(get_macs / tg / VALU_FLOOR_MACS_PER_S, 4),
                            "hbm_bytes": G * 2 * k * L, "plan": rt.plans["get"]},
        "issue_peak_gf_macs_per_s": float(f"{VALU_FLOOR_MACS_PER_S:.4g}"),
        "note": "issue_frac against the one bit-sliced VALU floor (ISSUE_PER_S x MACS_PER_INST_BS); kernel durations "
                "of the same command under rocprofv3 in profiles/r06/"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32, help="coded pieces per encode pass")
    ap.add_argument("--gens", type=int, default=16, help="resident generations (512 MiB: HBM-cold)")
    ap.add_argument("--per-generation", action="store_true",
                    help="one launch per generation per step (rounds 1-2 headline) instead of one grouped launch "
                         "over all resident generations")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the secondary measurements")
    ap.add_argument("--overlap", choices=("elim", "elim_sync", "elim_only", "copy", "get"), default="elim",
                    help="pipelined round trip: what step i + 1's encode runs beside (RoundTripStep)")
    ap.add_argument("--serial-roundtrip", action="store_true",
                    help="encoders and decoders on one context (stream): no encode of step i + 1 beside step i's "
                         "GetPieces (rounds 4-5 step)")
    ap.add_argument("--no-encode-decode", action="store_true",
                    help="skip the encode_decode round trip (PMC runs of the headline launch alone)")
    args = ap.parse_args()

    from kodr_amd import dist as kdist
    rank, world, local = kdist.world()

    # CPU baselines first, before this process touches the GPU and before the
    # process group starts (rank 0; at N > 1 a shorter sample): the encode
    # (value's unit) and kodr's decode, which make the round trip's baseline
    cpu = cpu_dec = None
    if rank == 0 and not args.no_cpu_baseline:
        secs = args.cpu_seconds if world == 1 else min(args.cpu_seconds, 3.0)
        cpu = cpu_baseline(secs)
        if not args.no_encode_decode:
            cpu_dec = cpu_baseline_decode(secs * 0.6)

    import numpy as np
    import torch  # plumbing: process group + shared HIP runtime
    import torch.distributed as dist

    # KODR_BENCH_REHEARSE=1: rehearsal of the N>1 path on a one-GPU box (every
    # rank on device 0, gloo instead of RCCL).  Never used for reported numbers.
    rehearse = os.environ.get("KODR_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo", init_method="env://")
        else:
            dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))

    from kodr_amd import device as kdev
    from kodr_amd import errors
    from kodr_amd._lib import last_launch_plan, lib

    L_ = lib()
    ctx = kdev.Context(local)
    k, L, B, G = K_PIECES, L_BYTES, args.batch, args.gens

    rng = np.random.default_rng(0x6B6F6472 + rank)
    hs = HeadlineStep(ctx, L_, errors, k, L, B, G, grouped=not args.per_generation, rng=rng)
    encs, dV, dOut = hs.encs, hs.dV, hs.dOut
    construct_ms, grouped, per_step, step = hs.construct_ms, hs.grouped, hs.per_step, hs.step

    def barrier():
        ctx.synchronize()
        if world > 1:
            dist.barrier()
        ctx.synchronize()

    extras = {"construct_ms_per_generation": round(construct_ms, 3)}
    # ---- value: the metric's encode + decode round trip (configs[1] encode +
    # configs[2] decode) over the G resident generations: W warmup + K timed
    # steps between barriers, max over ranks
    # (--no-encode-decode: the encode leg alone, for the PMC passes of tools/)
    ed = None
    if not args.no_encode_decode:
        # the decoders on a context of their own (own stream): the pipelined
        # round trip (RoundTripStep); --serial-roundtrip keeps every call on ctx
        dctx = ctx if args.serial_roundtrip else kdev.Context(local)
        elim0 = dctx.elim_stats()
        rt = RoundTripStep(ctx, L_, errors, encs, k, L, rng, dctx=dctx, overlap=args.overlap)

        def rt_barrier():
            rt.synchronize()
            if world > 1:
                dist.barrier()
            rt.synchronize()

        t_rt, n_warm_rt = run_timed(rt.step, args.steps, args.warmup, rt_barrier, WARM_S, phase=rt.begin_phase)
        warm_encodes = rt.encodes_before_phase
        elim1 = dctx.elim_stats()
        ed = roundtrip_block(t_rt, args.steps, args.warmup, n_warm_rt, rt.units(), world, kdist, device="cuda")
        ed["us_per_generation"] = round(ed["ms_per_step"] / G * 1e3, 2)
        ed["payload_MBps"] = round(world * args.steps * G * k * L / (ed["ms_per_step"] * args.steps / 1e3) / 1e6, 1)
        ed["wall_s"] = round(t_rt, 4)
        legs_in_step = roundtrip_kernels(rt, k, L)
        rt_ok = rt.decoded_ok()
        rt_n = rt.n
        rt_pipelined = rt.pipelined
        rt_overlap = rt.overlap if rt.pipelined else None
        # the elimination routes of every decoder of the warmup and timed steps
        # (rlnc_ctx_elim_stats): host_after_gpu counts the launches that left a
        # batch to kodr's algorithm on the host
        elim_routes = {key: elim1[key] - elim0[key] for key in elim0}
        rt.close()
        if dctx is not ctx:
            dctx.close()
        # The legs: in the pipelined step the encode shares the GPU with the
        # elimination and the twin copy, so its event time is not the kernel's.
        # The same round trip run in series right after (rounds 4-5's step,
        # every call on ctx; one untimed step, the GPU being warm) times each
        # leg alone in the step as it occurs; the roofline prices that encode.
        n_warm_serial = 0
        if rt_pipelined:
            rs = RoundTripStep(ctx, L_, errors, encs, k, L, rng)
            _, n_warm_serial = run_timed(rs.step, args.steps, 1, barrier, 0.0, phase=rs.begin_phase)
            legs = roundtrip_kernels(rs, k, L)
            rs.close()
            legs["pipelined_in_step"] = {key: {"avg_us": v["avg_us"]} for key, v in legs_in_step.items()
                                         if isinstance(v, dict) and "avg_us" in v}
        else:
            legs = legs_in_step
        legs["serial_warmup_steps"] = n_warm_serial
        # the hardware anchor: VALU instructions per launch from the committed
        # PMC pass of this command (tools/pmc_valu.py) over the SIMDs' VALU
        # issue capacity at the nominal 2.4 GHz during the leg's launch
        pv = pmc_valu(G, k, L)
        for leg in ("encode_launch", "get_pieces_call"):
            if pv and leg in pv:
                q, t_leg = pv[leg], legs[leg]["avg_us"] * 1e-6
                busy = round(q["valu_insts_per_launch"] * 2 / (1024 * 2.4e9 * t_leg), 4)
                sp = q.get("serial_phase") or {}
                legs[leg]["valu"] = {
                    "insts_per_launch": q["valu_insts_per_launch"],
                    "busy_at_nominal_clock": busy,
                    # the PMC pass's own launches of the same (serial) phase,
                    # with their rocprof durations: the like-for-like check
                    "busy_at_nominal_clock_pmc": sp.get("valu_busy_at_nominal_clock"),
                    "line_over_pmc": (round(busy / sp["valu_busy_at_nominal_clock"], 4)
                                      if sp.get("valu_busy_at_nominal_clock") else None),
                    "busy_at_measured_clock_pmc": sp.get("valu_busy_at_measured_clock",
                                                         q.get("valu_busy_at_measured_clock")),
                    "clock_ghz_pmc": q.get("clock_ghz"),
                    "source": pmc_valu_file(G, k, L)}

    # W warmup steps, but never fewer than one pass over the G generations (no
    # generation is first touched inside the timed region) and never less than
    # WARM_S of back-to-back work: after a load step the MI355X's clocks dip
    # for ~30 ms (a grouped launch goes 242 -> 338 -> 230 us,
    # profiles/r02/warm/), so the timed steps start at the sustained rate
    # whatever --warmup says
    n_warm = 0
    tw0 = time.perf_counter()
    while n_warm < max(args.warmup, 1 if grouped else G) or (time.perf_counter() - tw0 < WARM_S and n_warm < 20000):
        step(n_warm)
        n_warm += 1
        if n_warm % 8 == 0:
            ctx.synchronize()      # keep the host's clock on the device's work
    barrier()
    e0, e1 = ctx.event(), ctx.event()
    t0 = time.perf_counter()
    ctx.record(e0)
    for i in range(args.steps):
        step(i)
    ctx.record(e1)
    ms_dev = kdev.Context.elapsed_ms(e0, e1)
    plan = last_launch_plan()      # the timed launch's kernel instance (pinned by tests/test_gpu_headline.py)
    barrier()
    wall = time.perf_counter() - t0
    t_local = ms_dev / 1e3
    t_max = kdist.max_over_ranks(t_local, device="cuda")

    unit_bytes = setbytes(k, L)
    value = kdist.aggregate_rate(args.steps * per_step * B, unit_bytes, t_max, world)
    t_launch = t_local / args.steps
    # Roofline of the dominant kernel, per launch (one launch = one step):
    #  hbm:   the bytes a launch must move -- the generation once, B vectors
    #         in, B pieces out -- over the launch time, against 8 TB/s.  (kodr's
    #         SetBytes x B, the unit of `value`, counts the generation once per
    #         piece, so it is not an HBM byte count: B pieces share one read.)
    #  issue: GF MACs per second against the VALU floor of the bit-sliced
    #         method, the bound that binds at B >= 9 (Roofline).
    algo_bytes = per_step * B * unit_bytes
    compulsory = per_step * (k * L + B * k + B * L)
    achieved = compulsory / t_launch / 1e9
    macs = per_step * B * k * L
    bs = plan["kernel"] == 2


    if not args.no_extras and rank == 0:
        extras.update(run_extras(ctx, L_, errors, encs, dV, dOut, B, k, L, rng))
    if world > 1 and not args.no_extras:
        try:
            c5 = run_relay(HipRelayEngine(ctx, L_, errors, encs[0]), k, L, rng, torch, dist, kdist)
        except Exception as e:  # secondary measurement: never lose the headline line
            c5 = {"error": repr(e)[:300]}
        if rank == 0:
            extras["c5_encode_relay_recode"] = c5

    hs.close()

    if rank == 0 and ed is None:  # tools/ PMC passes: the encode leg alone
        print(json.dumps({"metric": "encode leg only (--no-encode-decode)", "value": round(value, 1),
                          "ms_per_step": round(t_max / args.steps * 1e3, 5), "plan": plan,
                          "avg_launch_us": round(t_launch * 1e6, 3)}), flush=True)
    elif rank == 0:
        enc_macs = G * rt_n * k * L
        te = legs["encode_launch"]["avg_us"] / 1e6
        step_s = ed["ms_per_step"] / 1e3
        gfbs_macs_step = enc_macs + G * k * k * L
        line = {
            "metric": "coded MB/s device-resident, Full-RLNC encode+decode, 32M/256 pieces @1/2/4/8 GPU",
            "value": ed["value"],
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ed["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded uniform random bytes and coding vectors)",
            "config": {"workload": (f"Full RLNC encode+decode round trip, 32 MiB generations / 256 pieces (BASELINE "
                                    f"configs[1] encode + configs[2] decode), device-resident: a step = {G} resident "
                                    f"generations x (k + 2 = {k + 2} coded pieces in one grouped encode launch, a "
                                    "fresh decoder each fed them in one batched AddPiece call (GPU elimination), one "
                                    "grouped GetPieces)"
                                    + (f"; pipelined (overlap {rt_overlap}): step i + 1's encode (encoders' stream) "
                                       "queued beside step i's elimination and twin copy (decoders' stream)"
                                       if rt_pipelined else "")
                                    + "; value in kodr units: (k + 2) x SetBytes (encoder bench) + DecodableLen "
                                      "(decoder bench) per generation"),
                       "value_covers": "encode+decode",
                       "piece_count": k, "piece_size": L, "generations_per_step": G,
                       "coded_pieces_per_generation_per_step": k + 2, "resident_generations": G,
                       "pipelined": rt_pipelined, "overlap": rt_overlap,
                       "parallelism": f"generation-sharded x{world}"},
            "roofline": {"bound": "valu", "achieved": float(f"{enc_macs / te:.4g}"),
                         "peak": float(f"{VALU_FLOOR_MACS_PER_S:.4g}"), "unit": "GF-MAC/s",
                         "frac": round(enc_macs / te / VALU_FLOOR_MACS_PER_S, 4),
                         "traffic": pmc_traffic(k + 2, k, L, G),
                         "traffic_source": pmc_traffic_file(k + 2, k, L, G),
                         "kernel": "gf_bs_kernel",
                         "avg_launch_us": round(te * 1e6, 2),
                         "legs": legs,
                         "step_share": {"gf_bs_macs_per_step": gfbs_macs_step,
                                        "gf_macs_per_s": float(f"{gfbs_macs_step / step_s:.4g}"),
                                        "frac": round(gfbs_macs_step / step_s / VALU_FLOOR_MACS_PER_S, 4),
                                        "note": "both gf_bs launches of a step (encode + GetPieces) over the whole "
                                                "step time: the kernel's rate with every other leg counted against it"},
                         "hbm": {"achieved_GBps": round(legs["encode_launch"]["hbm_bytes"] / te / 1e9, 1),
                                 "peak_GBps": HBM_PEAK_GBS,
                                 "frac": round(legs["encode_launch"]["hbm_bytes"] / te / 1e9 / HBM_PEAK_GBS, 4)},
                         "note": "the round trip's dominant kernel is gf_bs_kernel (the grouped encode launch, k + 2 "
                                 "pieces of 16 generations, and the grouped GetPieces, together ~89 % of a step's GPU "
                                 "time): 258 GF MACs per generation byte read, so neither HBM (hbm.frac) nor MFMA (a "
                                 "byte-field product) bounds it; SURVEY 8(d) prices decode against the VALU ceiling. "
                                 "achieved/frac: the round trip's encode launch (HIP events around it) in the same "
                                 "round trip run in series right after the timed (pipelined) steps, against the "
                                 "bit-sliced method's VALU issue floor; legs: every leg of that serial run, "
                                 "legs.pipelined_in_step: the timed steps' in-step event times; legs.*.valu: the "
                                 "hardware VALU-busy anchor from the committed PMC pass"},
            "cpu_baseline": (cpu_baseline_roundtrip(cpu, cpu_dec) if cpu is not None and cpu_dec is not None
                             else None),
            "roundtrip": {"us_per_generation": ed["us_per_generation"], "payload_MBps": ed["payload_MBps"],
                          "warmup_steps_run": ed["warmup_steps_run"],
                          "units_per_step_per_rank": ed["units_per_step_per_rank"],
                          "warmup_encodes_run": warm_encodes,
                          "roundtrip_ok": rt_ok, "elimination_routes": elim_routes},
            "encode": {
                "value": round(value, 1), "unit": "MB/s", "ms_per_step": round(t_max / args.steps * 1e3, 5),
                "workload": ("Full RLNC encode (BASELINE configs[1]), 32 MiB generation / 256 pieces; "
                             + (f"a step = {B} coded pieces of each of the {G} resident generations in one grouped "
                                "launch" if grouped else
                                f"a step = {B} coded pieces of one generation (rotating over {G})")
                             + "; kodr units: SetBytes per coded piece; same protocol (steps, warmup, barriers, "
                               "max over ranks)"),
                "coded_pieces_per_generation_per_step": B, "generations_per_step": per_step,
                "coded_pieces_per_step": per_step * B,
                "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                             "traffic": pmc_traffic(B, k, L, per_step),
                             "kernel": kernel_name(plan),
                             "plan": plan,
                             "traffic_source": pmc_traffic_file(B, k, L, per_step),
                             "hbm_bytes_per_launch": compulsory,
                             "avg_launch_us": round(t_launch * 1e6, 3),
                             "warmup_launches": n_warm, "generations_per_launch": per_step,
                             "issue": {"achieved_gf_macs_per_s": float(f"{macs / t_launch:.4g}"),
                                       "peak_gf_macs_per_s": float(f"{VALU_FLOOR_MACS_PER_S:.4g}"),
                                       "frac": round(macs / t_launch / VALU_FLOOR_MACS_PER_S, 4) if bs else None,
                                       "gf_macs_per_launch": macs},
                             "kodr_setbytes_per_launch": algo_bytes,
                             "note": "achieved/frac: the launch's compulsory HBM bytes (per generation: the "
                                     "generation once + B vectors + B pieces) / launch time / 8 TB/s; traffic: "
                                     "PMC-measured HBM bytes per launch (profiles/, FETCH_SIZE x2 + WRITE_SIZE); "
                                     "issue: GF MACs/s against the bit-sliced method's VALU floor"},
                "cpu_baseline": cpu,
                "wall_s": round(wall, 4),
            },
            "wall_s": ed["wall_s"],
        }
        if extras:
            line["extras"] = extras
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


WARM_S = 0.08


def kernel_name(plan):
    """The kernel a launch plan names (rlnc_last_launch_plan: the library's last launch)."""
    return {1: "gf_gemm_kernel", 2: "gf_bs_kernel", 3: "gf_gemv_kernel"}.get(plan["kernel"], "?")


def pmc_traffic_file(B, k, L, G=1):
    name = f"pmc_traffic_B{B}_k{k}_L{L}.json" if G == 1 else f"pmc_traffic_G{G}_B{B}_k{k}_L{L}.json"
    return "profiles/" + name


def pmc_valu_file(G, k, L):
    return f"profiles/pmc_valu_G{G}_k{k}_L{L}.json"


def pmc_valu(G, k, L):
    """VALU instructions per launch of the round trip's two gf_bs_kernel legs
    from the committed rocprofv3 --pmc summary (tools/pmc_valu.py)."""
    path = os.path.join(ROOT, pmc_valu_file(G, k, L))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def pmc_traffic(B, k, L, G=1):
    """HBM bytes per launch of this exact configuration, from the committed
    rocprofv3 --pmc summary (tools/profile_bench.sh: separate FETCH_SIZE and
    WRITE_SIZE passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM)."""
    path = os.path.join(ROOT, pmc_traffic_file(B, k, L, G))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


class HipRelayEngine:
    """The engine's side of the config-5 relay hop (C ABI on the GPU): k
    coded pieces of the rank's generation as wire rows with device-drawn
    vectors, and a recoder built on the rows received."""

    def __init__(self, ctx, L_, errors, enc):
        self.ctx, self.L_, self.errors, self.enc = ctx, L_, errors, enc

    def encode_wire(self, send, count, pitch):
        self.errors.check(self.L_.rlnc_encoder_coded_wire_device(self.enc, count, send.data_ptr(), pitch))

    def recode(self, recv, n, k, clen, pitch, dR, count, out):
        import ctypes
        rh = ctypes.c_void_p()
        self.errors.check(self.L_.rlnc_recoder_create_device(self.ctx.handle, recv.data_ptr(), n, clen, pitch, k,
                                                             ctypes.byref(rh)))
        self.errors.check(self.L_.rlnc_recoder_coded_pieces_device(rh, dR, count, out.data_ptr(), pitch))
        self.L_.rlnc_recoder_destroy(rh)

    def upload(self, R, torch):
        t = torch.from_numpy(R.reshape(-1)).to("cuda")
        return t, t.data_ptr()

    def synchronize(self):
        self.ctx.synchronize()


def run_relay(engine, k, L, rng, torch, dist, kdist, device="cuda", reps=6, keep=False, self_p2p=False):
    """BASELINE config 5 on N GPUs: every rank encodes k coded pieces of its
    generation (wire layout, kodr_amd.dist.wire_pitch), ring-shifts them to
    rank+1 over RCCL/xGMI, and recodes the k pieces it received.  Returns
    per-phase times (max over ranks); keep=True also returns the last
    repetition's buffers (tests check them against the oracle); self_p2p
    runs the exchange through the P2P ops even with one rank (GPU test)."""
    import numpy as np
    clen = k + L
    pitch = kdist.wire_pitch(k, L)
    send = torch.zeros(k * pitch, dtype=torch.uint8, device=device)
    recv = torch.empty_like(send)
    out = torch.zeros_like(send)
    Rv = rng.integers(0, 256, (k, k), dtype=np.uint8)
    Rkeep, dR = engine.upload(Rv, torch)
    times = {"encode": [], "exchange": [], "recode": []}
    for rep in range(reps):
        engine.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        engine.encode_wire(send, k, pitch)     # k wire rows [vector | piece]
        engine.synchronize()
        t1 = time.perf_counter()
        kdist.ring_shift(send, recv, self_p2p=self_p2p)
        if device == "cuda":
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        engine.recode(recv, k, k, clen, pitch, dR, k, out)
        engine.synchronize()
        t3 = time.perf_counter()
        if rep > 0:
            times["encode"].append(t1 - t0)
            times["exchange"].append(t2 - t1)
            times["recode"].append(t3 - t2)
    res = {}
    for name, ts in times.items():
        res[name + "_ms"] = round(kdist.max_over_ranks(min(ts), device=device) * 1e3, 4)
    res["exchange_GBps_per_link"] = round(k * pitch / (res["exchange_ms"] / 1e3) / 1e9, 2)
    # whole-job relay rate: every rank's k recoded pieces (kodr SetBytes (n+1)(k+L),
    # benches/full/recoder_test.go:53) over the slowest rank's encode + exchange + recode
    t_hop = (res["encode_ms"] + res["exchange_ms"] + res["recode_ms"]) / 1e3
    res["relay_recoded_MBps"] = round(kdist.aggregate_rate(k, (k + 1) * clen, t_hop, dist.get_world_size()), 1)
    res["note"] = "recode includes staging the received rows into the recoder (one D2D copy)"
    if keep:
        return res, {"send": send.cpu().numpy().reshape(k, pitch), "recv": recv.cpu().numpy().reshape(k, pitch),
                     "out": out.cpu().numpy().reshape(k, pitch), "R": Rv, "pitch": pitch, "clen": clen}
    return res


def two_streams(L_, errors, k, L, rng, batches=(1, 32), gens=16, steps=200):
    """Independent generations encoded from two contexts (two HIP streams)
    at once, steps alternating between them: the launch gap and the ramp of
    one stream's kernel overlap the other's.  Wall time over the steps, both
    streams drained; not the headline (per-kernel durations overlap)."""
    import ctypes
    import numpy as np
    from kodr_amd import device as kdev
    u8p = ctypes.POINTER(ctypes.c_uint8)
    ctxs = [kdev.Context(0), kdev.Context(0)]
    encs = [[], []]
    for g in range(gens):
        data = rng.integers(0, 256, k * L, dtype=np.uint8)
        h = ctypes.c_void_p()
        errors.check(L_.rlnc_encoder_create(ctxs[g % 2].handle, 0, data.ctypes.data_as(u8p), k, L, ctypes.byref(h)))
        encs[g % 2].append(h)
    res = {}
    for b in batches:
        V = rng.integers(0, 256, (b, k), dtype=np.uint8)
        bufs = []
        for c in ctxs:
            dv, do = c.alloc(V.nbytes), c.alloc(b * L)
            c.h2d(dv, V)
            bufs.append((dv, do))

        def step(i):
            s = i & 1
            errors.check(L_.rlnc_encoder_coded_pieces_device(encs[s][(i >> 1) % len(encs[s])], bufs[s][0], b,
                                                             bufs[s][1], L))
        for i in range(20):
            step(i)
        for c in ctxs:
            c.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        for c in ctxs:
            c.synchronize()
        dt = (time.perf_counter() - t0) / steps
        res[str(b)] = {"us_per_pass": round(dt * 1e6, 2), "coded_MBps": round(b * setbytes(k, L) / dt / 1e6, 1),
                       "generation_read_GBps": round(k * L / dt / 1e9, 1)}
        for c, (dv, do) in zip(ctxs, bufs):
            c.free(dv)
            c.free(do)
    for c, es in zip(ctxs, encs):
        for h in es:
            L_.rlnc_encoder_destroy(h)
        c.close()
    return res


def run_extras(ctx, L_, errors, encs, dV, dOut, B, k, L, rng):
    """Secondary measurements (not the headline): MALL-hot encode, full
    decode of 32 MiB/256 from device-resident pieces, host-path encode."""
    import ctypes
    import numpy as np
    from kodr_amd import device as kdev
    out = {}
    # MALL-hot: one generation re-read every step
    e0, e1 = ctx.event(), ctx.event()
    for i in range(10):
        L_.rlnc_encoder_coded_pieces_device(encs[0], dV, B, dOut, L)
    ctx.record(e0)
    for i in range(100):
        errors.check(L_.rlnc_encoder_coded_pieces_device(encs[0], dV, B, dOut, L))
    ctx.record(e1)
    t = kdev.Context.elapsed_ms(e0, e1) / 1e3 / 100
    out["encode_mall_hot_MBps"] = round(B * setbytes(k, L) / t / 1e6, 1)
    # coded pieces per pass: B = 1 is pure streaming, large B is VALU-bound
    sweep = {}
    Vs = rng.integers(0, 256, (k, k), dtype=np.uint8)
    dVs, dOs = ctx.alloc(Vs.nbytes), ctx.alloc(k * L)
    ctx.h2d(dVs, Vs)
    for b in (1, 2, 4, 8, 16, 32, 64, 256):
        iters = 40 if b <= 32 else 10
        for i in range(3):
            errors.check(L_.rlnc_encoder_coded_pieces_device(encs[i % len(encs)], dVs, b, dOs, L))
        ctx.record(e0)
        for i in range(iters):
            errors.check(L_.rlnc_encoder_coded_pieces_device(encs[i % len(encs)], dVs, b, dOs, L))
        ctx.record(e1)
        tb = kdev.Context.elapsed_ms(e0, e1) / 1e3 / iters
        sweep[str(b)] = {"us_per_pass": round(tb * 1e6, 2), "coded_MBps": round(b * setbytes(k, L) / tb / 1e6, 1),
                         "hbm_GBps": round((k * L + b * (k + L)) / tb / 1e9, 1)}
    out["encode_batch_sweep"] = sweep
    ctx.free(dVs)
    ctx.free(dOs)
    # coded pieces in wire layout with device-drawn vectors
    W = k + L
    dWire = ctx.alloc((k + 2) * W)
    for i in range(3):
        errors.check(L_.rlnc_encoder_coded_wire_device(encs[i % len(encs)], B, dWire, W))
    ctx.record(e0)
    for i in range(40):
        errors.check(L_.rlnc_encoder_coded_wire_device(encs[i % len(encs)], B, dWire, W))
    ctx.record(e1)
    tw = kdev.Context.elapsed_ms(e0, e1) / 1e3 / 40
    out["encode_wire_device_rng_MBps"] = round(B * setbytes(k, L) / tw / 1e6, 1)
    # decode C2: k + 2 wire rows on the device -> one batched AddPiece call + GetPieces
    n = k + 2
    dDec = ctx.alloc(k * L)

    def c2_wire(rep):  # fresh vectors per decode (one seed per rep)
        L_.rlnc_encoder_seed(encs[0], 7 + rep)
        errors.check(L_.rlnc_encoder_coded_wire_device(encs[0], n, dWire, W))

    # ~6 % of random k = 256 vector sets have a singular 16 x 16 leading block
    # somewhere (panel-local pivoting in the GPU elimination), and those take
    # kodr's host route after the launch: seeds 7 and 8 are two such sets, so
    # a single fixed seed would time only that path
    out["c2_decode"] = time_decode(ctx, L_, errors, dWire, n, W, k, L, dDec, reps=12, regen=c2_wire, warm=1)
    td = out["c2_decode"]["s"]
    out["c2_decode"]["MBps_decodable_len"] = round(k * (k + L) / td / 1e6, 1)
    out["c2_decode"]["gf_macs_per_s"] = float(f"{k * k * L / td:.4g}")
    # the same decode fed one AddPiece call per piece
    Vd = ctx.d2h(dWire, n * W).reshape(n, W)[:, :k].copy()
    vptr = [Vd[i].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) for i in range(n)]  # (no ctypes object building timed)
    pptr = [ctypes.c_void_p(dWire + i * W + k) for i in range(n)]
    times_pw = []
    for rep in range(3):
        dh = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
        t0 = time.perf_counter()
        for i in range(n):
            st = L_.rlnc_decoder_add_piece_device_borrowed(dh, vptr[i], k, pptr[i], L)
            if st == 3:
                break
            errors.check(st)
        errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
        ctx.synchronize()
        times_pw.append(time.perf_counter() - t0)
        L_.rlnc_decoder_destroy(dh)
    out["c2_decode"]["piecewise_s"] = round(min(times_pw), 6)
    # verify the decode against the resident generation
    pitch = ctypes.c_size_t()
    dp = L_.rlnc_encoder_device_pieces(encs[0], ctypes.byref(pitch))
    a = ctx.d2h(dDec, k * L)
    b = ctx.d2h(dp, k * pitch.value).reshape(k, pitch.value)[:, :L].reshape(-1)
    out["c2_decode"]["roundtrip_ok"] = bool(np.array_equal(a, b))
    ctx.free(dWire)
    ctx.free(dDec)
    out["c2_decode_grouped"] = c2_decode_grouped(ctx, L_, errors, encs, k, L)
    out["north_star_grouped_encode"] = grouped_encode(ctx, L_, errors, encs, k, L, rng)
    out["c2_recode"] = recode_c2(ctx, L_, errors, encs[0], k, L, rng)
    out["c5_encode_recode_one_gpu"] = c5_one_gpu(ctx, L_, errors, encs[:8], k, L, rng)
    out["c5_encode_recode_one_gpu_grouped"] = c5_one_gpu_grouped(ctx, L_, errors, encs[:8], k, L, rng)
    out["c4_systematic_decode"] = c4_decode(ctx, L_, errors, rng)
    out["batched_decode_elimination"] = batched_elim(ctx, L_, errors, rng)
    out["batched_decode_elimination_rounds"] = batched_elim_rounds(ctx, L_, errors, rng)
    out["c2_decode_piecewise_grouped"] = piecewise_grouped(ctx, L_, errors, encs, k, L)
    out["c1_roundtrip"] = c1_roundtrip(ctx, L_, errors, rng)
    out["encode_two_streams"] = two_streams(L_, errors, k, L, rng)
    out["host_path"] = host_roundtrip(ctx, L_, errors, k, L, rng)
    out["host_path_registered"] = host_roundtrip(ctx, L_, errors, k, L, rng, pinned=True)
    return out


# One issue ceiling for every GF product kernel, one derivation: 1024 SIMDs at
# 2.4 GHz issuing a wave instruction every 2.3 cycles with 4 waves per SIMD
# (profiles/r01/dispatch_probe.log, straight-line XOR3), times the GF MACs per
# VALU instruction of the kernel's method.  gf_bs_kernel: per coefficient and
# 2 KiB wave slice 8 XOR3 (7.97 on average) + the row's 26 table instructions
# shared by 8 output rows, 2048 MACs -> 195 T MAC/s (the VALU floor; its
# v_readlane and SALU are left out, so this is an upper bound).
# gf_gemm_kernel: per coefficient and 256 B 3 v_perm + 1.5 XOR3 + the
# selector share (0.5) -> 55 T MAC/s.
ISSUE_PER_S = 1024 * 2.4e9 / 2.3
MACS_PER_INST_BS = 2048 / (7.97 + 26 / 8)
MACS_PER_INST_PERM = 256 / 5
VALU_FLOOR_MACS_PER_S = ISSUE_PER_S * MACS_PER_INST_BS


def grouped_encode(ctx, L_, errors, encs, k, L, rng, iters=50):
    """North-star shape (BASELINE north_star: encode of a 32 MiB/256
    generation at >= 70 % of HBM read): `count` coded pieces of each of the G
    resident generations in ONE launch (rlnc_encoder_group_coded_pieces_device,
    gf_gemm_kernel with a generation grid dimension), so the launch and ramp
    are paid once per G x 32 MiB.  HIP events on the context stream."""
    from kodr_amd._lib import last_launch_plan
    import ctypes
    import numpy as np
    from kodr_amd import device as kdev
    G = len(encs)
    arr = (ctypes.c_void_p * G)(*[e.value for e in encs])
    res = {"generations_per_launch": G}
    e0, e1 = ctx.event(), ctx.event()
    for count in (1, 2, 4, 8, 16, 32, 64):
        iters_c = iters if count <= 8 else 10
        V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
        dV, dO = ctx.alloc(V.nbytes), ctx.alloc(G * count * L)
        ctx.h2d(dV, V)
        for i in range(5):
            errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, count, dO, L))
        ctx.record(e0)
        for i in range(iters_c):
            errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, count, dO, L))
        ctx.record(e1)
        t = kdev.Context.elapsed_ms(e0, e1) / 1e3 / iters_c
        hbm = G * (k * L + count * (k + L))
        # prepared encoders: the bit-sliced launch from 5 pieces (capi.cpp kGroupBsMinRows)
        res[str(count)] = {"kernel": kernel_name(last_launch_plan()) + " (grouped)",
                           "us_per_launch": round(t * 1e6, 2), "us_per_generation": round(t / G * 1e6, 3),
                           "coded_MBps": round(G * count * setbytes(k, L) / t / 1e6, 1),
                           "hbm_GBps": round(hbm / t / 1e9, 1),
                           "hbm_frac": round(hbm / t / 1e9 / HBM_PEAK_GBS, 4)}
        ctx.free(dV)
        ctx.free(dO)
    res["note"] = ("hbm = generation read once per piece batch + vectors + pieces, per launch; "
                   "count=1 is the north-star shape (one coded piece per 32 MiB generation)")
    return res


def recode_c2(ctx, L_, errors, enc, k, L, rng, iters=40):
    """Full recode at 32 MiB/256 (kodr README.md:111: 1,074.82 MB/s on one
    i7 core): a recoder holding n = k coded pieces (wire rows drawn by the
    engine's encoder), B recoded pieces per call, kodr's SetBytes
    (n+1)(k+L) per piece (benches/full/recoder_test.go:53).  The recoder's
    bit-sliced twin is built at construction (rlnc_recoder_prepare)."""
    from kodr_amd._lib import last_launch_plan
    import ctypes
    import numpy as np
    from kodr_amd import device as kdev
    n, clen = k, k + L
    pitch = (clen + 255) // 256 * 256
    dW = ctx.alloc(n * pitch)
    errors.check(L_.rlnc_encoder_coded_wire_device(enc, n, dW, pitch))
    rh = ctypes.c_void_p()
    ctx.synchronize()
    t0 = time.perf_counter()
    errors.check(L_.rlnc_recoder_create_device(ctx.handle, dW, n, clen, pitch, k, ctypes.byref(rh)))
    errors.check(L_.rlnc_recoder_prepare(rh))
    ctx.synchronize()
    res = {"construct_ms": round((time.perf_counter() - t0) * 1e3, 3), "unit_bytes": (n + 1) * clen,
           "kodr_published_MBps": 1074.82}
    e0, e1 = ctx.event(), ctx.event()
    R = rng.integers(0, 256, (256, n), dtype=np.uint8)
    dR, dO = ctx.alloc(R.nbytes), ctx.alloc(256 * pitch)
    ctx.h2d(dR, R)
    for b in (1, 32, 256):
        it = iters if b <= 32 else 10
        for i in range(3):
            errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, b, dO, pitch))
        ctx.record(e0)
        for i in range(it):
            errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, b, dO, pitch))
        ctx.record(e1)
        t = kdev.Context.elapsed_ms(e0, e1) / 1e3 / it
        res[str(b)] = {"us_per_call": round(t * 1e6, 2), "recoded_MBps": round(b * (n + 1) * clen / t / 1e6, 1),
                       "kernel": kernel_name(last_launch_plan())}
    L_.rlnc_recoder_destroy(rh)
    for p in (dW, dR, dO):
        ctx.free(p)
    return res


def c5_one_gpu(ctx, L_, errors, encs, k, L, rng, reps=3):
    """BASELINE config 5's per-GPU work on one GPU: for each of 8 resident
    32 MiB/256 generations, k coded pieces in wire layout (device-drawn
    vectors), a recoder built on those rows, k recoded pieces.  The N>1 run adds
    the RCCL ring shift between the two (extras.c5_encode_relay_recode)."""
    import ctypes
    import numpy as np
    clen = k + L
    pitch = (clen + 255) // 256 * 256
    G = len(encs)
    dW, dO = ctx.alloc(k * pitch), ctx.alloc(k * pitch)
    R = rng.integers(0, 256, (k, k), dtype=np.uint8)
    dR = ctx.alloc(R.nbytes)
    ctx.h2d(dR, R)
    best = None
    for rep in range(reps):
        ctx.synchronize()
        t0 = time.perf_counter()
        for e in encs:
            errors.check(L_.rlnc_encoder_coded_wire_device(e, k, dW, pitch))
            rh = ctypes.c_void_p()
            errors.check(L_.rlnc_recoder_create_device(ctx.handle, dW, k, clen, pitch, k, ctypes.byref(rh)))
            errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, k, dO, pitch))
            L_.rlnc_recoder_destroy(rh)   # synchronises the stream
        ctx.synchronize()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    for p in (dW, dO, dR):
        ctx.free(p)
    units = G * k * (setbytes(k, L) + (k + 1) * clen)
    return {"generations": G, "ms": round(best * 1e3, 3), "ms_per_generation": round(best / G * 1e3, 3),
            "coded_plus_recoded_MBps": round(units / best / 1e6, 1),
            "note": "per generation: k encoded + k recoded pieces, kodr SetBytes units for both; host wall time, "
                    "recoder construction (D2D copy of the received rows + twin) included"}


def c5_one_gpu_grouped(ctx, L_, errors, encs, k, L, rng, reps=3):
    """c5_one_gpu with grouped launches: k coded pieces of all 8 generations
    in ONE encode launch (rlnc_encoder_group_coded_pieces_device, written into
    the pieces' columns of the wire rows), a recoder per generation on its
    rows, and k recoded pieces of all 8 in ONE recode launch
    (rlnc_recoder_group_coded_pieces_device).  The coding vectors are random
    host bytes uploaded before the timed region, into both the contiguous
    vector block and the wire rows (64 KiB per generation); the recoded
    output is spot-checked for one generation (two recoded rows: vector part
    R x V and piece part vector x P, numpy GF(2^8) in _gf_vecmat)."""
    import ctypes
    import numpy as np
    clen = k + L
    pitch = (clen + 255) // 256 * 256
    G = len(encs)
    V = rng.integers(0, 256, (G, k, k), dtype=np.uint8)
    R = rng.integers(0, 256, (G, k, k), dtype=np.uint8)
    dV, dR = ctx.alloc(V.nbytes), ctx.alloc(R.nbytes)
    ctx.h2d(dV, V)
    ctx.h2d(dR, R)
    dW, dO = ctx.alloc(G * k * pitch), ctx.alloc(G * k * pitch)
    wire = np.zeros((G * k, pitch), np.uint8)
    wire[:, :k] = V.reshape(G * k, k)
    ctx.h2d(dW, wire)
    del wire
    earr = (ctypes.c_void_p * G)(*[e.value for e in encs])
    best = None
    for rep in range(reps):
        ctx.synchronize()
        t0 = time.perf_counter()
        errors.check(L_.rlnc_encoder_group_coded_pieces_device(earr, G, dV, k, dW + k, pitch))
        recs = []
        for g in range(G):
            rh = ctypes.c_void_p()
            errors.check(L_.rlnc_recoder_create_device(ctx.handle, dW + g * k * pitch, k, clen, pitch, k,
                                                       ctypes.byref(rh)))
            recs.append(rh)
        errors.check(L_.rlnc_recoder_group_coded_pieces_device((ctypes.c_void_p * G)(*[r.value for r in recs]), G,
                                                               dR, k, dO, pitch))
        ctx.synchronize()
        t = time.perf_counter() - t0
        for rh in recs:
            L_.rlnc_recoder_destroy(rh)
        best = t if best is None else min(best, t)
    # generation G-1, recoded rows 0 and k-1: vector part = R x V, and the row
    # is a codeword of the generation (piece = vector x P), numpy GF(2^8)
    pp = ctypes.c_size_t()
    dp = L_.rlnc_encoder_device_pieces(encs[G - 1], ctypes.byref(pp))
    ok = None
    if dp:
        P = ctx.d2h(dp, k * pp.value).reshape(k, pp.value)[:, :L]
        got = ctx.d2h(dO + (G - 1) * k * pitch, k * pitch).reshape(k, pitch)[:, :clen]
        ok = True
        for i in (0, k - 1):
            vec = _gf_vecmat(R[G - 1, i], V[G - 1])
            ok = ok and bool(np.array_equal(got[i, :k], vec)) and bool(np.array_equal(got[i, k:], _gf_vecmat(vec, P)))
    for p_ in (dV, dR, dW, dO):
        ctx.free(p_)
    units = G * k * (setbytes(k, L) + (k + 1) * clen)
    return {"generations": G, "ms": round(best * 1e3, 3), "ms_per_generation": round(best / G * 1e3, 3),
            "coded_plus_recoded_MBps": round(units / best / 1e6, 1), "recoded_rows_ok": ok,
            "note": "one grouped encode launch + G recoder constructions (D2D copy + twin) + one grouped recode "
                    "launch; host wall time; parity of both grouped entry points in tests/test_gpu_headline.py"}


def _gf_vecmat(v, M):
    """v (n bytes) x M (n x w bytes) over GF(2^8), poly 0x11D (gf256.go:15-44),
    with numpy log/exp tables: a spot check of engine output, not a baseline."""
    import numpy as np
    exp = np.zeros(512, np.int32)
    log = np.zeros(256, np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    exp[255:510] = exp[:255]
    acc = np.zeros(M.shape[1], np.int32)
    for j, c in enumerate(np.asarray(v, np.int32)):
        if c:
            row = M[j].astype(np.int32)
            acc ^= np.where(row != 0, exp[(log[row] + log[c]) % 255], 0)
    return acc.astype(np.uint8)


def c2_decode_grouped(ctx, L_, errors, encs, k, L, reps=3):
    """BASELINE configs[2] over many generations: each of the G resident
    generations' encoders writes k + 2 coded wire rows (device-drawn vectors),
    then G fresh decoders take them in ONE batched AddPiece call
    (rlnc_decoders_add_pieces_gpu: one elimination launch) and ONE grouped
    GetPieces call (rlnc_decoders_get_pieces_device: one bit-sliced launch).
    Wall time per generation, decoder construction outside the timed region
    (as kodr's decoder bench, benches/full/decoder_test.go); outputs checked
    against the generations' resident pieces."""
    import ctypes
    import numpy as np
    G, n, W = len(encs), k + 2, k + L
    wires = []
    for g, e in enumerate(encs):
        L_.rlnc_encoder_seed(e, 1000 + g)
        dw = ctx.alloc(n * W)
        errors.check(L_.rlnc_encoder_coded_wire_device(e, n, dw, W))
        wires.append(dw)
    dO = ctx.alloc(G * k * L)
    best, ok = None, True
    for rep in range(reps):
        decs = []
        for g in range(G):
            h = ctypes.c_void_p()
            errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
            decs.append(h)
        darr = (ctypes.c_void_p * G)(*[x.value for x in decs])
        ctx.synchronize()
        t0 = time.perf_counter()
        cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
        errors.check(L_.rlnc_decoders_add_pieces_gpu(darr, G, (ctypes.c_void_p * G)(*wires),
                                                     (ctypes.c_size_t * G)(*([n] * G)), W, L, cons, sts))
        t1 = time.perf_counter()
        errors.check(L_.rlnc_decoders_get_pieces_device(darr, G, dO, L))
        ctx.synchronize()
        t2 = time.perf_counter()
        ok = ok and all(s_ in (0, 3) for s_ in sts) and all(L_.rlnc_decoder_is_decoded(x) for x in decs)
        for x in decs:
            L_.rlnc_decoder_destroy(x)
        if best is None or t2 - t0 < best[0]:
            best = (t2 - t0, t1 - t0, t2 - t1)
    pitch = ctypes.c_size_t()
    for g in (0, G - 1):
        dp = L_.rlnc_encoder_device_pieces(encs[g], ctypes.byref(pitch))
        a = ctx.d2h(dO + g * k * L, k * L)
        b = ctx.d2h(dp, k * pitch.value).reshape(k, pitch.value)[:, :L].reshape(-1)
        ok = ok and bool(np.array_equal(a, b))
    for d in wires:
        ctx.free(d)
    ctx.free(dO)
    t, ta, tg = best
    return {"generations": G, "ms": round(t * 1e3, 3), "add_ms": round(ta * 1e3, 3), "get_ms": round(tg * 1e3, 3),
            "us_per_generation": round(t / G * 1e6, 1),
            "MBps_decodable_len": round(G * k * (k + L) / t / 1e6, 1),
            "gf_macs_per_s": float(f"{G * k * k * L / t:.4g}"), "roundtrip_ok": ok,
            "note": "wall time of one batched AddPiece + one grouped GetPieces over G generations"}


def batched_elim(ctx, L_, errors, rng, k=256, G=32, L=256, reps=3):
    """Batched AddPiece on G fresh decoders (k + 2 device wire rows each,
    short pieces so the coefficient side dominates): host elimination
    (rlnc_decoder_add_pieces per decoder) against one GPU launch
    (rlnc_decoders_add_pieces_gpu, gf_elim.hip: a workgroup per decoder)."""
    import ctypes
    import numpy as np
    n = k + 2
    pitch = (k + L + 15) // 16 * 16
    bufs = []
    for g in range(G):
        rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
        d = ctx.alloc(rows.nbytes)
        ctx.h2d(d, rows)
        bufs.append(d)
    res = {"k": k, "generations": G, "piece_len": L}
    for mode in ("host", "gpu"):
        best, ok = None, True
        for rep in range(reps):
            decs = []
            for g in range(G):
                h = ctypes.c_void_p()
                errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
                decs.append(h)
            ctx.synchronize()
            t0 = time.perf_counter()
            if mode == "host":
                with host_elimination(ctx):
                    for g in range(G):
                        c = ctypes.c_size_t()
                        st = L_.rlnc_decoder_add_pieces(decs[g], bufs[g], n, pitch, L, 1, ctypes.byref(c))
                        ok = ok and st in (0, 3)
            else:
                cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
                errors.check(L_.rlnc_decoders_add_pieces_gpu((ctypes.c_void_p * G)(*[x.value for x in decs]), G,
                                                             (ctypes.c_void_p * G)(*bufs), (ctypes.c_size_t * G)(*([n] * G)),
                                                             pitch, L, cons, sts))
                ok = ok and all(s_ in (0, 3) for s_ in sts)
            ctx.synchronize()
            t = time.perf_counter() - t0
            ok = ok and all(L_.rlnc_decoder_is_decoded(x) for x in decs)
            for x in decs:
                L_.rlnc_decoder_destroy(x)
            best = t if best is None else min(best, t)
        res[mode + "_ms"] = round(best * 1e3, 3)
        res[mode + "_ok"] = ok
    res["gpu_speedup"] = round(res["host_ms"] / res["gpu_ms"], 2)
    for d in bufs:
        ctx.free(d)
    return res


def piecewise_grouped(ctx, L_, errors, encs, k, L, reps=2):
    """C2 fed the way kodr's decoder is (one AddPiece per piece,
    full/decoder.go:50-66), for every resident generation at once: G decoders
    take k device wire rows each, round-robin, one rlnc_decoder_add_piece_device_borrowed
    call per piece (lazy AddPiece queues them), then the queues are eliminated
    either by ONE rlnc_decoders_flush_gpu call (GPU elimination) or by each
    decoder's own state read (host); two more pieces per generation follow
    (refused once decoded, used where the first k were dependent), and one
    grouped GetPieces decodes all.
    ctypes arguments are built outside the timed region (a Go caller pays no
    such cost); best of reps."""
    import ctypes
    import numpy as np
    G, W, n = len(encs), k + L, k + 2
    earr = (ctypes.c_void_p * G)(*[e.value for e in encs])
    dW = ctx.alloc(G * n * W)
    dO = ctx.alloc(G * k * L)
    res = {"generations": G}
    for mode in ("host", "gpu"):
        best, ok = None, True
        for rep in range(reps + 1):
            errors.check(L_.rlnc_encoder_group_coded_wire_device(earr, G, n, dW, W))
            vec = ctx.d2h(dW, G * n * W).reshape(G * n, W)[:, :k].copy()
            decs = []
            for g in range(G):
                h = ctypes.c_void_p()
                errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
                decs.append(h)
            darr = (ctypes.c_void_p * G)(*[x.value for x in decs])
            add = L_.rlnc_decoder_add_piece_device_borrowed
            args = [(decs[g], vec[g * n + i].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), dW + (g * n + i) * W + k)
                    for i in range(n) for g in range(G)]
            ctx.synchronize()
            t0 = time.perf_counter()
            for h, v, p_ in args[:k * G]:
                if add(h, v, k, p_, L) != 0:
                    ok = False
            t1 = time.perf_counter()
            if mode == "gpu":
                errors.check(L_.rlnc_decoders_flush_gpu(darr, G))
            else:
                with host_elimination(ctx):
                    for h in decs:
                        L_.rlnc_decoder_is_decoded(h)
            t2 = time.perf_counter()
            for h, v, p_ in args[k * G:]:
                if add(h, v, k, p_, L) not in (0, 3):
                    ok = False
            errors.check(L_.rlnc_decoders_get_pieces_device(darr, G, dO, L))
            ctx.synchronize()
            t3 = time.perf_counter()
            ok = ok and all(L_.rlnc_decoder_is_decoded(x) for x in decs)
            for x in decs:
                L_.rlnc_decoder_destroy(x)
            if rep and (best is None or t3 - t0 < best[0]):
                best = (t3 - t0, t1 - t0, t2 - t1, t3 - t2)
        pitch = ctypes.c_size_t()
        for g in (0, G - 1):
            dp = L_.rlnc_encoder_device_pieces(encs[g], ctypes.byref(pitch))
            a = ctx.d2h(dO + g * k * L, k * L)
            b = ctx.d2h(dp, k * pitch.value).reshape(k, pitch.value)[:, :L].reshape(-1)
            ok = ok and bool(np.array_equal(a, b))
        t, t_add, t_flush, t_rest = best
        res[mode] = {"ms": round(t * 1e3, 3), "us_per_generation": round(t / G * 1e6, 1),
                     "add_calls_us_per_generation": round(t_add / G * 1e6, 1),
                     "flush_us_per_generation": round(t_flush / G * 1e6, 1),
                     "spare_adds_and_get_us_per_generation": round(t_rest / G * 1e6, 1), "roundtrip_ok": ok}
    # the whole piecewise decode is the like-for-like comparison: the host flush
    # (IsDecoded) leaves the gather of the queued pieces to the next data call,
    # the GPU flush does it in the flush
    res["decode_speedup"] = round(res["host"]["us_per_generation"] / res["gpu"]["us_per_generation"], 2)
    res["note"] = ("k AddPiece calls per generation (device pieces, round-robin over the generations), the queued "
                   "eliminations flushed by one rlnc_decoders_flush_gpu (gpu) or by each decoder's IsDecoded (host), "
                   "2 more AddPiece calls per generation, one grouped GetPieces; wall time")
    ctx.free(dW)
    ctx.free(dO)
    return res


def batched_elim_rounds(ctx, L_, errors, rng, k=256, G=32, L=256, rounds=4, reps=3):
    """Batched AddPiece on G decoders fed in `rounds` batches each (k + 2
    device wire rows split evenly, short pieces so the coefficient side
    dominates): host elimination per decoder (rlnc_decoder_add_pieces)
    against one rlnc_decoders_add_pieces_gpu call per round.  After the first
    round the decoders are no longer fresh: their batches are eliminated on
    the GPU from [held coefficient rows ; batch vectors] (continued decoders,
    DecoderCore::load_continued).  Wall time per round, best of reps."""
    import ctypes
    import numpy as np
    n = k + 2
    pitch = (k + L + 15) // 16 * 16
    cuts = [round(i * n / rounds) for i in range(rounds + 1)]
    bufs = []
    for g in range(G):
        rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
        d = ctx.alloc(rows.nbytes)
        ctx.h2d(d, rows)
        bufs.append(d)
    res = {"k": k, "generations": G, "piece_len": L, "rows_per_round": [cuts[i + 1] - cuts[i] for i in range(rounds)]}
    for mode in ("host", "gpu"):
        best, ok = None, True
        for rep in range(reps):
            decs = []
            for g in range(G):
                h = ctypes.c_void_p()
                errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
                decs.append(h)
            ts = []
            for r in range(rounds):
                ctx.synchronize()
                t0 = time.perf_counter()
                cnt = cuts[r + 1] - cuts[r]
                if mode == "host":
                    with host_elimination(ctx):
                        for g in range(G):
                            c = ctypes.c_size_t()
                            st = L_.rlnc_decoder_add_pieces(decs[g], bufs[g] + cuts[r] * pitch, cnt, pitch, L, 1,
                                                            ctypes.byref(c))
                            ok = ok and st in (0, 3)
                else:
                    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
                    errors.check(L_.rlnc_decoders_add_pieces_gpu(
                        (ctypes.c_void_p * G)(*[x.value for x in decs]), G,
                        (ctypes.c_void_p * G)(*[b + cuts[r] * pitch for b in bufs]),
                        (ctypes.c_size_t * G)(*([cnt] * G)), pitch, L, cons, sts))
                    ok = ok and all(s_ in (0, 3) for s_ in sts)
                ctx.synchronize()
                ts.append(time.perf_counter() - t0)
            ok = ok and all(L_.rlnc_decoder_is_decoded(x) for x in decs)
            for x in decs:
                L_.rlnc_decoder_destroy(x)
            if best is None or sum(ts) < sum(best):
                best = ts
        res[mode + "_ms_per_round"] = [round(t * 1e3, 3) for t in best]
        res[mode + "_ms"] = round(sum(best) * 1e3, 3)
        res[mode + "_ok"] = ok
    res["gpu_speedup"] = round(res["host_ms"] / res["gpu_ms"], 2)
    for d in bufs:
        ctx.free(d)
    return res


def time_decode(ctx, L_, errors, dWire, n, W, k, L, dDec, reps=3, regen=None, warm=0):
    """One batched AddPiece call over n device wire rows + GetPieces into
    device memory (synchronous), best of reps fresh decoders.  regen(rep), if
    given, rewrites the wire rows before each rep (untimed): fresh coding
    vectors per decode, as kodr draws them per piece (data.go:90-95); the
    medians over the reps are reported beside the best.  warm: untimed reps
    first (regen(-1), ...: other vector sets), so that the timed reps do not
    pay the process's first launch of this shape's kernels."""
    import ctypes
    import statistics
    from kodr_amd._codec import elim_stats
    best = None
    adds, tots = [], []
    routes = {}
    for rep in range(-warm, reps):
        if regen is not None:
            regen(rep)
            ctx.synchronize()
        dh = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
        consumed = ctypes.c_size_t()
        t0 = time.perf_counter()
        st = L_.rlnc_decoder_add_pieces(dh, dWire, n, W, L, 1, ctypes.byref(consumed))
        if st != 3:
            errors.check(st)
        t1 = time.perf_counter()
        errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
        ctx.synchronize()
        t2 = time.perf_counter()
        gf, cp = ctypes.c_size_t(), ctypes.c_size_t()
        errors.check(L_.rlnc_decoder_apply_stats(dh, ctypes.byref(gf), ctypes.byref(cp)))
        decoded = bool(L_.rlnc_decoder_is_decoded(dh))
        bs = bool(L_.rlnc_decoder_last_apply_bitsliced(dh))
        recv = L_.rlnc_decoder_received(dh)
        if rep >= 0:
            for key, v in elim_stats(dh).items():  # which route eliminated the batch (rlnc_decoder_elim_stats)
                routes[key] = routes.get(key, 0) + v
        L_.rlnc_decoder_destroy(dh)
        if rep < 0:
            continue
        adds.append(t1 - t0)
        tots.append(t2 - t0)
        if best is None or t2 - t0 < best["s"]:
            best = {"s": round(t2 - t0, 6), "add_s": round(t1 - t0, 6), "get_s": round(t2 - t1, 6),
                    "gf_rows": gf.value, "copy_rows": cp.value, "received": recv, "decoded": decoded, "bs": bs}
    if reps > 3:
        best["reps"] = reps
        best["s_median"] = round(statistics.median(tots), 6)
        best["add_s_median"] = round(statistics.median(adds), 6)
        best["add_s_max"] = round(max(adds), 6)
        best["add_s_reps"] = [round(x * 1e6, 1) for x in adds]  # us, in rep order (each rep a fresh vector set)
    best["elimination_routes"] = routes
    macs = best["gf_rows"] * best["received"] * L
    best["apply_gf_macs"] = macs
    best["apply_gf_macs_per_s"] = float(f"{macs / best['get_s']:.4g}")
    bs = best.pop("bs")
    mpi = MACS_PER_INST_BS if bs else MACS_PER_INST_PERM
    best["apply_kernel"] = "gf_bs_kernel" if bs else "gf_gemm_kernel"
    best["issue_ceiling_macs_per_s"] = float(f"{ISSUE_PER_S * mpi:.4g}")
    return best


def c4_decode(ctx, L_, errors, rng):
    """BASELINE config 4 (systematic 16 MiB/128): 10% of the systematic pieces
    lost and replaced by coded ones.  The decoder copies the systematic rows and
    runs GF work only for the missing ones; the same generation
    decoded from coded pieces only is timed beside it.  kodr: 1.821 s
    (README.md:188)."""
    import ctypes
    import numpy as np
    k, L = 128, 131072
    W = k + L
    data = rng.integers(0, 256, k * L, dtype=np.uint8)
    eh = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 1, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                        ctypes.byref(eh)))
    errors.check(L_.rlnc_encoder_seed(eh, 4))
    n = 2 * k + 4
    dAll = ctx.alloc(n * W)
    errors.check(L_.rlnc_encoder_coded_wire_device(eh, n, dAll, W))
    rows = ctx.d2h(dAll, n * W).reshape(n, W)
    res_enc = c4_encode(ctx, L_, errors, data, k, L)
    lost = set(rng.choice(k, k // 10, replace=False).tolist())
    keep = [i for i in range(k) if i not in lost] + list(range(k, n))
    kept = np.ascontiguousarray(rows[keep])
    coded = np.ascontiguousarray(rows[k:])
    dKept, dCoded, dDec = ctx.alloc(kept.nbytes), ctx.alloc(coded.nbytes), ctx.alloc(k * L)
    ctx.h2d(dKept, kept)
    ctx.h2d(dCoded, coded)
    res = {"encode": res_enc, "lost_systematic": len(lost)}
    res["systematic"] = time_decode(ctx, L_, errors, dKept, kept.shape[0], W, k, L, dDec)
    ok = bool(np.array_equal(ctx.d2h(dDec, k * L), data))
    res["full_coded_only"] = time_decode(ctx, L_, errors, dCoded, coded.shape[0], W, k, L, dDec)
    ok = ok and bool(np.array_equal(ctx.d2h(dDec, k * L), data))
    res["roundtrip_ok"] = ok
    res["speedup_vs_full"] = round(res["full_coded_only"]["s"] / res["systematic"]["s"], 2)
    for p in (dAll, dKept, dCoded, dDec):
        ctx.free(p)
    L_.rlnc_encoder_destroy(eh)
    return res


def c4_encode(ctx, L_, errors, data, k, L, B=32, iters=40):
    """Systematic encode at BASELINE config 4 (16 MiB/128), device-resident
    wire rows with device-drawn vectors: the first k pieces are e_i ++ P_i
    copies (systematic/encoder.go:83-96), later ones coded, B per call.
    kodr's SetBytes per piece: S + (k+L) (benches/systematic/encoder_test.go:44)."""
    import ctypes
    from kodr_amd import device as kdev
    W = k + L
    unit = k * L + W
    dW = ctx.alloc(k * W)
    e0, e1 = ctx.event(), ctx.event()
    t_sys = []
    for rep in range(3):
        eh = ctypes.c_void_p()
        errors.check(L_.rlnc_encoder_create(ctx.handle, 1, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k,
                                            L, ctypes.byref(eh)))
        ctx.synchronize()
        ctx.record(e0)
        errors.check(L_.rlnc_encoder_coded_wire_device(eh, k, dW, W))   # the k systematic pieces
        ctx.record(e1)
        ctx.synchronize()
        t_sys.append(kdev.Context.elapsed_ms(e0, e1) / 1e3)
        if rep < 2:
            L_.rlnc_encoder_destroy(eh)
    for i in range(3):
        errors.check(L_.rlnc_encoder_coded_wire_device(eh, B, dW, W))
    ctx.record(e0)
    for i in range(iters):
        errors.check(L_.rlnc_encoder_coded_wire_device(eh, B, dW, W))
    ctx.record(e1)
    t_cod = kdev.Context.elapsed_ms(e0, e1) / 1e3 / iters
    L_.rlnc_encoder_destroy(eh)
    ctx.free(dW)
    ts = min(t_sys)
    return {"systematic_k_pieces_us": round(ts * 1e6, 2), "systematic_MBps": round(k * unit / ts / 1e6, 1),
            "coded_B": B, "coded_us_per_call": round(t_cod * 1e6, 2),
            "coded_MBps": round(B * unit / t_cod / 1e6, 1),
            "first_2k_pieces_MBps": round(2 * k * unit / (ts + k / B * t_cod) / 1e6, 1),
            "unit_bytes": unit}


def _page_aligned(np, n):
    buf = np.empty((n + 4095) // 4096 * 4096 + 4096, np.uint8)
    off = (-buf.ctypes.data) % 4096
    return buf[off:off + n]


def host_roundtrip(ctx, L_, errors, k, L, rng, pinned=False):
    """The path as it sits in a service: 32 MiB from host memory -> device
    generation -> k+2 coded pieces back to host (batches of 16, then all in one
    call) -> decoder fed
    from host buffers in one batched AddPiece call -> decoded pieces back to
    host.  Pageable host buffers staged through pinned chunks inside the
    library, synchronous C-ABI calls (PCIe-inclusive)."""
    import ctypes
    import numpy as np
    u8p = ctypes.POINTER(ctypes.c_uint8)
    n = k + 2
    if pinned:  # caller-owned page-locked slabs (rlnc_host_register)
        data, V = _page_aligned(np, k * L), _page_aligned(np, n * k).reshape(n, k)
        wire, outp = _page_aligned(np, n * (k + L)).reshape(n, k + L), _page_aligned(np, k * L)
        for a in (data, V, wire, outp):
            ctx.register(a)
        data[:] = rng.integers(0, 256, k * L, dtype=np.uint8)
        V[:] = rng.integers(0, 256, (n, k), dtype=np.uint8)
    else:
        data = rng.integers(0, 256, k * L, dtype=np.uint8)
        V = rng.integers(0, 256, (n, k), dtype=np.uint8)
        wire = np.empty((n, k + L), np.uint8)
        outp = np.empty(k * L, np.uint8)
    t0 = time.perf_counter()
    eh = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create_with_piece_count(ctx.handle, 0, data.ctypes.data_as(u8p), data.size, k,
                                                        ctypes.byref(eh)))
    t1 = time.perf_counter()
    for i in range(0, n, 16):
        b = min(16, n - i)
        errors.check(L_.rlnc_encoder_coded_pieces(eh, V[i:i + b].ctypes.data_as(u8p), b,
                                                 wire[i:i + b].ctypes.data_as(u8p)))
    t2 = time.perf_counter()
    # the same k+2 pieces in one call (the library pipelines sub-batches: the
    # D2H of one overlaps the kernel of the next when the buffer is pinned)
    tc0 = time.perf_counter()
    errors.check(L_.rlnc_encoder_coded_pieces(eh, V.ctypes.data_as(u8p), n, wire.ctypes.data_as(u8p)))
    tc1 = time.perf_counter()
    # decode alone: the k + 2 host wire rows into a fresh decoder (one batched
    # AddPiece: H2D of the rows, elimination) and the k decoded pieces back
    dh = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
    td0 = time.perf_counter()
    consumed = ctypes.c_size_t()
    st = L_.rlnc_decoder_add_pieces(dh, wire.ctypes.data_as(u8p), n, k + L, L, 0, ctypes.byref(consumed))
    if st != 3:
        errors.check(st)
    td1 = time.perf_counter()
    errors.check(L_.rlnc_decoder_get_pieces(dh, outp.ctypes.data_as(u8p)))
    td2 = time.perf_counter()
    ok = bool(np.array_equal(outp, data))
    L_.rlnc_decoder_destroy(dh)
    L_.rlnc_encoder_destroy(eh)
    if pinned:
        for a in (data, V, wire, outp):
            ctx.unregister(a)
    t_dec = td2 - td0
    t_rt = (t1 - t0) + (tc1 - tc0) + t_dec
    # PCIe floor of the round trip at the box's 56 GB/s each way (profiles/r01/pcie.log):
    # the generation up, k + 2 wire rows down, the same rows up, k pieces down
    floor = (k * L + 2 * n * (k + L) + k * L) / 56e9
    return {"upload_ms": round((t1 - t0) * 1e3, 3),
            "encode_k+2_to_host_ms": round((t2 - t1) * 1e3, 3),
            "encode_coded_MBps_incl_pcie": round(n * setbytes(k, L) / (t2 - t1) / 1e6, 1),
            "encode_k+2_one_call_ms": round((tc1 - tc0) * 1e3, 3),
            "encode_one_call_pcie_GBps": round(n * (k + L) / (tc1 - tc0) / 1e9, 1),
            "decode_from_host_ms": round(t_dec * 1e3, 3),
            "decode_add_pieces_ms": round((td1 - td0) * 1e3, 3),
            "decode_get_pieces_to_host_ms": round((td2 - td1) * 1e3, 3),
            "roundtrip_host_resident_ms": round(t_rt * 1e3, 3),
            "roundtrip_pcie_floor_ms": round(floor * 1e3, 3),
            "roundtrip_payload_MBps": round(k * L / t_rt / 1e6, 1),
            "roundtrip_ok": ok,
            "note": "one generation: upload (create from host data), k + 2 coded pieces to host in one call, "
                    "decode from those host rows (batched AddPiece + GetPieces to host); pcie floor = 4 transfers "
                    "of the generation's size at 56 GB/s"}


if __name__ == "__main__":
    main()
