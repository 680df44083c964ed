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


class OracleRelayEngine:
    """CPU stand-in for bench.HipRelayEngine: the same wire layout (rows of
    k + L bytes at kodr_amd.dist.wire_pitch) produced and recoded by the
    oracle, on CPU tensors."""

    def __init__(self, P, seed):
        self.P = P
        self.rng = np.random.default_rng(seed)

    def encode_wire(self, send, count, pitch):
        import oracle
        k, L = self.P.shape
        V = self.rng.integers(0, 256, (count, k), dtype=np.uint8)
        rows = send.numpy().reshape(-1, pitch)
        rows[:count, :k] = V
        rows[:count, k:k + L] = oracle.encode(self.P, V)

    def recode(self, recv, n, k, clen, pitch, R, count, out):
        import oracle
        src = recv.numpy().reshape(-1, pitch)[:n, :clen]
        out.numpy().reshape(-1, pitch)[:count, :clen] = oracle.recode(np.ascontiguousarray(src), k, R[:count])

    def upload(self, R, torch):
        return R, R

    def synchronize(self):
        pass


def _relay_worker(rank, ws, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    import bench
    import oracle
    from kodr_amd import dist as kd
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=ws)
    try:
        k, L = 16, 1000
        P = np.random.default_rng(200 + rank).integers(0, 256, (k, L), dtype=np.uint8)
        eng = OracleRelayEngine(P, 300 + rank)
        res, buf = bench.run_relay(eng, k, L, np.random.default_rng(7 + rank), torch, dist, kd, device="cpu",
                                   reps=2, keep=True)
        pitch, clen = buf["pitch"], buf["clen"]
        assert pitch == (k + L + 255) // 256 * 256 and clen == k + L
        sends = [None] * ws
        dist.all_gather_object(sends, buf["send"])
        prev = (rank - 1) % ws
        shifted = np.array_equal(buf["recv"], sends[prev])
        recoded = np.array_equal(buf["out"][:, :clen], oracle.recode(np.ascontiguousarray(buf["recv"][:, :clen]), k,
                                                                         buf["R"]))
        # the recoded rows decode the previous rank's generation
        d = oracle.Decoder(k)
        for row in buf["out"][:, :clen]:
            if d.add(row[:k], row[k:]) == 3:
                break
        Pp = np.random.default_rng(200 + prev).integers(0, 256, (k, L), dtype=np.uint8)
        decoded = d.is_decoded() and np.array_equal(np.stack([d.get_piece(i)[1] for i in range(k)]), Pp)
        q.put((rank, shifted, recoded, decoded, sorted(res)))
    finally:
        dist.destroy_process_group()


def test_bench_run_relay_two_ranks():
    # bench.py's own config-5 relay (run_relay: encode -> ring shift -> recode,
    # max-over-ranks timing, aggregate rate) with an oracle engine on CPU tensors
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_relay_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(ws))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, shifted, recoded, decoded, keys in res:
        assert shifted and recoded and decoded, rank
        assert {"encode_ms", "exchange_ms", "recode_ms", "relay_recoded_MBps"} <= set(keys)


def test_shard_generations_partition():
    from kodr_amd.dist import shard_generations
    for n in range(0, 20):
        for ws in range(1, 9):
            owned = [g for r in range(ws) for g in shard_generations(n, ws, r)]
            assert owned == list(range(n))


def _roundtrip_worker(rank, ws, port, q):
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    import bench
    import oracle
    from kodr_amd import dist as kd
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=ws)
    try:
        # bench.py's encode_decode protocol (run_timed + roundtrip_block) with a
        # CPU stand-in step: k + 2 coded pieces of this rank's generation by the
        # oracle, a fresh oracle decoder fed them; rank 1 is slower on purpose
        k, L = 8, 96
        P = np.random.default_rng(400 + rank).integers(0, 256, (k, L), dtype=np.uint8)
        rng = np.random.default_rng(500 + rank)
        seen = {"ok": True, "timed": 0}

        def step(i, timed):
            V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
            C = oracle.encode(P, V)
            d = oracle.Decoder(k)
            for j in range(k + 2):
                if d.add(V[j], C[j]) == 3:
                    break
            seen["ok"] &= d.is_decoded() and np.array_equal(np.stack([d.get_piece(j)[1] for j in range(k)]), P)
            seen["timed"] += int(timed)
            if rank == 1:
                time.sleep(0.01)

        units = 10_000_000 * (k + 2)  # stand-in units, large enough that the rounded value is exact
        t, n_warm = bench.run_timed(step, 5, 2, dist.barrier, 0.0)
        blk = bench.roundtrip_block(t, 5, 2, n_warm, units, ws, kd)
        q.put((rank, t, blk, seen["ok"], seen["timed"], n_warm))
    finally:
        dist.destroy_process_group()


def test_bench_roundtrip_block_two_ranks():
    # the encode_decode block at N = 2: every rank runs the round trip, the
    # time is the slowest rank's, the value aggregates both ranks' units
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_roundtrip_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(ws))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    t_max = max(r[1] for r in res)
    assert res[1][1] >= 0.05                                     # the slow rank's 5 x 10 ms
    for rank, t, blk, ok, timed, n_warm in res:
        assert ok and timed == 5 and n_warm == 2, rank
        assert blk["n_gpus"] == 2 and blk["steps"] == 5 and blk["warmup"] == 2
        assert blk["ms_per_step"] == pytest.approx(t_max / 5 * 1e3, rel=1e-4)
        assert blk["value"] == pytest.approx(2 * 5 * blk["units_per_step_per_rank"] / t_max / 1e6, rel=1e-3)
    assert res[0][2] == res[1][2]                                # one block, whatever the rank
