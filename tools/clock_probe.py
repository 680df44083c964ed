#!/usr/bin/env python3
"""The GPU's clock and power while grouped bit-sliced launches run back to
back: `amd-smi metric -c -p --json` sampled from a thread (each sample a
child process) during timed phases of B coded pieces of 16 resident 32 MiB /
256 generations per launch (bench.py's HeadlineStep), B from argv.  Prints
per phase the launch time and the median of the sampled clocks and power;
raw samples to argv[1].  usage: clock_probe.py OUT.jsonl B [B ...]"""
import json
import os
import re
import subprocess
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

samples = []
stop = False


def sampler():
    while not stop:
        t = time.time()
        try:
            r = subprocess.run(["amd-smi", "metric", "-g", "0", "-c", "-p", "--json"], capture_output=True, text=True,
                               timeout=5)
            samples.append((t, r.stdout))
        except Exception as e:  # noqa: BLE001
            samples.append((t, "ERR " + repr(e)))
        time.sleep(0.05)


def nums(txt, key):
    return [float(x) for x in re.findall(r'"%s"\s*:\s*\{\s*"value"\s*:\s*([0-9.]+)' % key, txt)]


def main():
    global stop
    out = sys.argv[1]
    Bs = [int(x) for x in sys.argv[2:]] or [32, 256]
    from kodr_amd import device as kdev, errors
    from kodr_amd._lib import lib
    ctx = kdev.Context(0)
    L_ = lib()
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    time.sleep(1.0)
    phases = [("idle0", None, time.time(), time.time())]
    rng = np.random.default_rng(1)
    hs = None
    for B in Bs:
        hs = bench.HeadlineStep(ctx, L_, errors, 256, 131072, B, 16, grouped=True, rng=rng)
        e0, e1 = ctx.event(), ctx.event()
        i = 0
        t0 = time.time()
        ctx.record(e0)
        while time.time() - t0 < 3.0:
            hs.step(i)
            i += 1
            if i % 4 == 0:
                ctx.synchronize()
        ctx.record(e1)
        ctx.synchronize()
        t1 = time.time()
        ms = kdev.Context.elapsed_ms(e0, e1)
        phases.append((f"B={B}", ms * 1e3 / i, t0, t1))
        hs.close()
        time.sleep(1.0)
        phases.append((f"idle_after_B={B}", None, t1, time.time()))
    stop = True
    th.join()
    with open(out, "w") as f:
        for t, s in samples:
            f.write(json.dumps({"t": t, "raw": s}) + "\n")
    print("first sample:", samples[0][1][:1500] if samples else None)
    for name, us, a, b in phases:
        sel = [s for t, s in samples if a + 0.3 <= t <= b]
        gfx = [v for s in sel for v in nums(s, "clk")[:1]]
        pw = [v for s in sel for v in nums(s, "socket_power")[:1]]
        print(f"{name:16s} launch {us if us is None else round(us, 1)} us; samples {len(sel)}; first clk value median "
              f"{np.median(gfx) if gfx else None}; socket power median {np.median(pw) if pw else None}")


if __name__ == "__main__":
    main()
