"""Multi-GPU plumbing for the batched-generations configuration.

Generations are independent (column-separable, no shared state), so the
engine shards whole generations over ranks, one process per GPU, with no
collective on the data path (weak scaling).  The one real exchange is the relay
hop of BASELINE config 5 ("encode+recode"): rank r encodes its generation and
forwards the coded pieces (wire layout, vector ++ piece) to rank r+1, which
recodes them -- a ring shift over xGMI via RCCL point-to-point.  RCCL has no
XOR reduction, so a generation is never row-sharded with an all-reduce.

torch.distributed is the transport only ("nccl" = RCCL on ROCm; "gloo" for the
CPU tests).
"""
import os


def world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_generations(n_generations, world_size, rank):
    """Contiguous block of generation indices owned by `rank`."""
    base, extra = divmod(n_generations, world_size)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def wire_pitch(k, L):
    """Row pitch of the engine's device wire rows (vector ++ piece, k + L
    bytes, CodedPiece.Flatten data.go:52-57) padded to the 256-byte alignment
    of its recoder and decoder rows (capi_internal.hpp kPitchAlign)."""
    return (k + L + 255) // 256 * 256


def ring_shift(send, recv, group=None, self_p2p=False):
    """Send `send` to rank+1 and receive into `recv` from rank-1 (one P2P step).
    With one rank the shift is a copy, unless self_p2p: then the same
    isend/irecv pair runs with the rank as its own peer (the GPU test that
    moves bytes through RCCL on a one-GPU box)."""
    import torch.distributed as dist
    rank, ws = dist.get_rank(group), dist.get_world_size(group)
    if ws == 1 and not self_p2p:
        recv.copy_(send)
        return
    if send.is_cuda and dist.get_backend(group) == "gloo":   # CPU-transport rehearsal
        s, r = send.cpu(), recv.cpu()
        ring_shift(s, r, group)
        recv.copy_(r)
        return
    ops = [dist.P2POp(dist.isend, send, (rank + 1) % ws, group),
           dist.P2POp(dist.irecv, recv, (rank - 1) % ws, group)]
    for r in dist.batch_isend_irecv(ops):
        r.wait()


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (the slowest rank times the job)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(units_per_rank, unit_bytes, seconds_max, world_size):
    """Whole-job throughput in 10^6 B/s: every rank's units over the slowest rank's time."""
    return world_size * units_per_rank * unit_bytes / seconds_max / 1e6
