"""Timeline of one gf_elim_mc4_kernel launch from a KODR_ELIM_DUMP file of a
-DKODR_ELIM_TIMING build (written by tools/elim_ab.py's last call, G = 1):
s_memrealtime stamps (10 ns) per workgroup in its 1 KiB of the T region --
chain [p] staged, [16 + p] block updated, [32 + p] S_p out, staging wave
[48 + p]; row workgroup [j] R_j / S_j in LDS, [16 + j] apply(j) done; [96]
entry, [97] tables in LDS.  usage: python tools/elim_mc4_stamps.py DUMP [k]"""
import sys

import numpy as np

k = int(sys.argv[2]) if len(sys.argv) > 2 else 256
raw = np.fromfile(sys.argv[1], dtype=np.uint8)
HDR = 4 * 256
NP = (k + 15) // 16
NRW = NP * 2
st = raw[HDR:HDR + k * k].view(np.uint64).reshape(-1, 128)[:NRW + 1]
t0 = min(int(st[x, 96]) for x in range(NRW + 1) if st[x, 96])
us = lambda v: (int(v) - t0) / 100.0  # 100 MHz
ch = st[NRW]
print(f"entry spread: {max(us(st[x, 96]) for x in range(NRW + 1)):.2f} us; chain tables {us(ch[97]):.2f}")
print("panel  staged  blk_upd  S_out   (chain)   rowwg0 R/S in  apply done  | last row wg apply done")
for p in range(NP):
    print(f"{p:5d} {us(ch[p]):7.2f} {us(ch[16 + p]):8.2f} {us(ch[32 + p]):7.2f}           "
          f"{us(st[0, p]):7.2f} {us(st[0, 16 + p]):10.2f}  | {max(us(st[x, 16 + p]) for x in range(NRW)):7.2f}")
print(f"last S_p out {us(ch[32 + NP - 1]):.2f} us; last apply {max(us(st[x, 16 + NP - 1]) for x in range(NRW)):.2f} us")
