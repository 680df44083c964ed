#!/usr/bin/env python3
"""Print per-kernel ISA statistics from a hipcc -save-temps .s file.

usage: tools/kernel_isa.py FILE.s [substring] [--dump]
"""
import re
import sys


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur:
            body.append(line)
            if "s_endpgm" in line:
                yield cur, body
                cur = None


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    for name, body in kernels(path):
        if sub not in name:
            continue
        text = "".join(body)
        stats = {k: len(re.findall(p, text)) for k, p in [
            ("lines", r"\n"), ("v_perm", r"v_perm_b32"), ("v_xor", r"v_xor|v_bitop3"),
            ("glb_load", r"global_load|buffer_load"), ("ds_read", r"ds_read"),
            ("scratch", r"scratch_|buffer_store_dword.*off"), ("waitcnt", r"s_waitcnt"),
            ("branches", r"s_cbranch")]}
        print(name[:90], stats)
        if "--dump" in sys.argv:
            print(text)


if __name__ == "__main__":
    main()
