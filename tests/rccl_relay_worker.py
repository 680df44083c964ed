"""Child process of tests/test_gpu_rccl.py: bench.py's config-5 relay
(run_relay: wire encode -> ring shift -> recode) on the GPU with a one-rank
RCCL process group whose ring shift runs the isend/irecv pair with the rank
as its own peer, so the bytes of the exchange move through RCCL.  Checks the
shifted rows, the recoded rows against the oracle and that they decode the
generation; prints one JSON line.  The oracle is the checker only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    import oracle
    from kodr_amd import device as kdev
    from kodr_amd import dist as kdist
    from kodr_amd import errors
    from kodr_amd._lib import lib
    import ctypes

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        k, L = int(sys.argv[1]), int(sys.argv[2])
        L_ = lib()
        ctx = kdev.Context(0)
        P = np.random.default_rng(11).integers(0, 256, (k, L), dtype=np.uint8)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        enc = ctypes.c_void_p()
        errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(u8p), k, L, ctypes.byref(enc)))
        eng = bench.HipRelayEngine(ctx, L_, errors, enc)
        res, buf = bench.run_relay(eng, k, L, np.random.default_rng(5), torch, dist, kdist, reps=3, keep=True,
                                   self_p2p=True)
        L_.rlnc_encoder_destroy(enc)
        clen = buf["clen"]
        send, recv, out = buf["send"], buf["recv"], buf["out"]
        # the sent rows are codewords of P: piece = vector x P
        codewords = np.array_equal(send[:, k:clen], oracle.encode(P, np.ascontiguousarray(send[:, :k])))
        shifted = np.array_equal(recv, send)
        recoded = np.array_equal(out[:, :clen], oracle.recode(np.ascontiguousarray(recv[:, :clen]), k, buf["R"]))
        d = oracle.Decoder(k)
        for row in out[:, :clen]:
            if d.add(row[:k], row[k:]) == 3:
                break
        decoded = bool(d.is_decoded()) and np.array_equal(np.stack([d.get_piece(i)[1] for i in range(k)]), P)
        print(json.dumps({"backend": dist.get_backend(), "codewords": bool(codewords), "shifted": bool(shifted),
                          "recoded": bool(recoded), "decoded": bool(decoded), "res": res}), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
