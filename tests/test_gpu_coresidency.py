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

The scenario runs in a child process (tests/gpu_child/coresidency.py) with
only its own streams: streams beyond GPU_MAX_HW_QUEUES (4 on the box) share
hardware queues, and in a long pytest session one of the context's streams
can land on the occupier's queue and wait for it whatever the library does
(57 ms, profiles/r05/coresidency/)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_elimination_beside_a_long_kernel_returns_early():
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_child", "coresidency.py")], capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(f"call {res['call_s'] * 1e3:.2f} ms; routes {res['routes']}")
    assert all(res["ok"]), res
    assert res["call_s"] <= 0.010, res
