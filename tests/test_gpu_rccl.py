"""The config-5 relay's RCCL leg on the GPU (kodr_amd/dist.py ring_shift,
bench.py run_relay).  The pool's boxes have one GPU and RCCL refuses two
ranks on one device (profiles/r03/rccl_same_gpu/), so the exchange runs in a
one-rank "nccl" process group with the rank as its own isend/irecv peer: the
same batch_isend_irecv code as at N > 1, the bytes moved by RCCL.  The
recoded rows are compared with the oracle (full/recoder.go:27-46) and decoded
back to the generation."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("k,L", [(16, 4096), (64, 65536)])
def test_relay_through_rccl_self_p2p(k, L):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_relay_worker.py"), str(k), str(L)],
                       env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [s for s in p.stdout.splitlines() if s.startswith("{")][-1]
    r = json.loads(line)
    assert r["backend"] == "nccl"
    assert r["codewords"] and r["shifted"] and r["recoded"] and r["decoded"], r
    assert r["res"]["exchange_ms"] > 0
