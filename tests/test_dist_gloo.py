"""world_size-2 tests of the multi-GPU plumbing on CPU (gloo).

They run the same code path as bench.py at N>1 -- generation sharding,
max-over-ranks timing, whole-job aggregation and the config-5 relay hop (ring
shift of wire-format coded pieces) -- with the CPU oracle standing in for the
GPU kernels as the producer/checker of the bytes that travel.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    import oracle
    from kodr_amd import dist as kd
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=ws)
    try:
        r, w, _ = kd.world()
        assert (r, w) == (rank, ws)
        gens = kd.shard_generations(5, ws, rank)
        # each rank encodes k coded pieces of its own generation (wire rows)
        k, L = 8, 64
        rng = np.random.default_rng(100 + rank)
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
        wire = np.concatenate([V, oracle.encode(P, V)], axis=1)
        send = torch.from_numpy(wire.copy())
        recv = torch.empty_like(send)
        kd.ring_shift(send, recv)
        # the receiver recodes what it got and decodes the neighbour's generation
        got = recv.numpy()
        R = rng.integers(0, 256, (k + 4, k + 2), dtype=np.uint8)
        rec = oracle.recode(got, k, R)
        d = oracle.Decoder(k)
        for row in rec:
            if d.add(row[:k], row[k:]) == 3:
                break
        dec = np.stack([d.get_piece(i)[1] for i in range(k)])
        # the neighbour's generation, regenerated from its seed
        prev = (rank - 1) % ws
        Pp = np.random.default_rng(100 + prev).integers(0, 256, (k, L), dtype=np.uint8)
        t = kd.max_over_ranks(0.5 + rank)
        q.put((rank, gens, bool(np.array_equal(dec, Pp)), t,
               kd.aggregate_rate(10, 1_000_000, t, ws)))
    finally:
        dist.destroy_process_group()


def test_two_rank_relay_and_aggregation():
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [[0, 1, 2], [3, 4]]      # sharding covers 0..4 once
    assert all(r[2] for r in res)                           # relay hop decodes exactly
    assert all(r[3] == pytest.approx(1.5) for r in res)     # max over ranks
    assert res[0][4] == pytest.approx(2 * 10 * 1e6 / 1.5 / 1e6)


def test_shard_generations_partition():
    from kodr_amd.dist import shard_generations
    for n in range(0, 20):
        for ws in range(1, 9):
            owned = [g for r in range(ws) for g in shard_generations(n, ws, r)]
            assert owned == list(range(n))
