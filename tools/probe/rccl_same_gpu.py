"""Can RCCL run the config-5 ring shift with two ranks on ONE GPU?  (The
one-GPU box cannot run the 8-GPU node's RCCL leg; this checks whether the
nccl backend at least executes kodr_amd.dist.ring_shift with both ranks on
device 0.)  Launch: torchrun --nproc-per-node 2 tools/probe/rccl_same_gpu.py.
Measurement/probe only."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kodr_amd import dist as kdist  # noqa: E402

rank, ws, _ = kdist.world()
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", 0))
n = 256 * kdist.wire_pitch(256, 131072)
send = torch.full((n,), rank + 1, dtype=torch.uint8, device="cuda")
recv = torch.zeros_like(send)
for _ in range(3):
    kdist.ring_shift(send, recv)
torch.cuda.synchronize()
ok = bool((recv == ((rank - 1) % ws) + 1).all().item())
ts = []
for _ in range(10):
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kdist.ring_shift(send, recv)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
t = kdist.max_over_ranks(min(ts), device="cuda")
if rank == 0:
    print(f"rccl ring_shift {ws} ranks on one GPU: ok={ok} {n / 2**20:.1f} MiB in {t * 1e3:.3f} ms "
          f"({n / t / 1e9:.1f} GB/s per rank)", flush=True)
dist.destroy_process_group()
