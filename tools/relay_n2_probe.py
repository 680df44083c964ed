#!/usr/bin/env python3
"""Why the config-5 relay's recode reads milliseconds in the N = 2 rehearsal
(two ranks on ONE GPU, gloo; bench.py KODR_BENCH_REHEARSE=1) against 0.21 ms
alone.  Launched like the rehearsal:

  KODR_BENCH_REHEARSE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 tools/relay_n2_probe.py

Rank 0 times the recode of bench.run_relay split into its three C ABI calls
(rlnc_recoder_create_device: the rows' 2D D2D copy + a stream sync;
rlnc_recoder_coded_pieces_device + sync; rlnc_recoder_destroy) while rank 1:
  idle          waits at the next barrier (its GPU context open, no work);
  recode        runs the same recode at the same moment;
  h2d_pageable  copies a pageable 33 MB host tensor to the GPU 4 times
                (what gloo's ring shift does at the end: recv.copy_(cpu));
  relay         bench.run_relay's own sequence on both ranks (encode, gloo
                ring shift, recode), every rank's split.
Rank 0 prints one JSON object: per scenario the min and median of each part
over the reps."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from kodr_amd import device as kdev  # noqa: E402
from kodr_amd import dist as kdist  # noqa: E402
from kodr_amd import errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

REPS = 8


def main():
    rank, world, _ = kdist.world()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="env://")
    L_ = lib()
    ctx = kdev.Context(0)
    k, L = bench.K_PIECES, bench.L_BYTES
    rng = np.random.default_rng(11 + rank)
    data = rng.integers(0, 256, k * L, dtype=np.uint8)
    enc = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                        ctypes.byref(enc)))
    eng = bench.HipRelayEngine(ctx, L_, errors, enc)
    clen, pitch = k + L, kdist.wire_pitch(k, L)
    send = torch.zeros(k * pitch, dtype=torch.uint8, device="cuda")
    recv = torch.empty_like(send)
    out = torch.zeros_like(send)
    _, dR = eng.upload(rng.integers(0, 256, (k, k), dtype=np.uint8), torch)
    eng.encode_wire(send, k, pitch)
    eng.encode_wire(recv, k, pitch)
    host = torch.empty(k * pitch, dtype=torch.uint8)   # pageable
    ctx.synchronize()

    def recode_split():
        rh = ctypes.c_void_p()
        t0 = time.perf_counter()
        errors.check(L_.rlnc_recoder_create_device(ctx.handle, recv.data_ptr(), k, clen, pitch, k, ctypes.byref(rh)))
        t1 = time.perf_counter()
        errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, k, out.data_ptr(), pitch))
        ctx.synchronize()
        t2 = time.perf_counter()
        L_.rlnc_recoder_destroy(rh)
        t3 = time.perf_counter()
        return {"create_ms": (t1 - t0) * 1e3, "product_ms": (t2 - t1) * 1e3, "destroy_ms": (t3 - t2) * 1e3,
                "recode_ms": (t3 - t0) * 1e3}

    res = {}
    for scen in ("idle", "recode", "h2d_pageable", "idle_again"):
        parts = []
        for rep in range(REPS):
            ctx.synchronize()
            torch.cuda.synchronize()
            dist.barrier()
            if rank == 0:
                parts.append(recode_split())
            elif scen == "recode":
                recode_split()
            elif scen == "h2d_pageable":
                for _ in range(4):
                    recv.copy_(host)
                torch.cuda.synchronize()
            dist.barrier()
        if rank == 0:
            res[scen] = {p: {"min": round(min(x[p] for x in parts), 4),
                             "median": round(statistics.median(x[p] for x in parts), 4)}
                         for p in parts[0]}
        print(f"rank {rank} {scen} done", flush=True)
    # bench.run_relay's sequence, with rank 0's recode split
    parts, exch, stamps = [], [], []
    for rep in range(REPS):
        eng.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        eng.encode_wire(send, k, pitch)
        eng.synchronize()
        t1 = time.perf_counter()
        kdist.ring_shift(send, recv)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        p = recode_split()
        t3 = time.perf_counter()
        exch.append((t2 - t1) * 1e3)
        parts.append(p)
        # host clock (CLOCK_MONOTONIC, one clock for both processes), ms
        stamps.append({"barrier_exit": t0 * 1e3, "encoded": t1 * 1e3, "exchanged": t2 * 1e3,
                       "created": (t2 * 1e3 + p["create_ms"]), "recoded": t3 * 1e3})
    mine = {p: {"min": round(min(x[p] for x in parts), 4), "median": round(statistics.median(x[p] for x in parts), 4)}
            for p in parts[0]}
    mine["exchange_ms"] = {"min": round(min(exch), 4), "median": round(statistics.median(exch), 4)}
    every = [None] * world
    dist.all_gather_object(every, {"split": mine, "stamps": stamps})
    if rank == 0:
        res["relay"] = {f"rank{r}": every[r]["split"] for r in range(world)}
        # per rep: every rank's events in ms after the earliest barrier exit
        tl = []
        for i in range(REPS):
            base = min(every[r]["stamps"][i]["barrier_exit"] for r in range(world))
            tl.append({f"rank{r}": {e: round(v - base, 3) for e, v in every[r]["stamps"][i].items()}
                       for r in range(world)})
        res["relay_timeline"] = tl
        print(json.dumps({"k": k, "L": L, "reps": REPS, "scenarios": res}), flush=True)
    dist.barrier()
    L_.rlnc_encoder_destroy(enc)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
