"""Summarise tools/probe/cu_map output: which blocks share a CU, and whether
the assignment follows block % 8 -> XCC and (block / 8) % 32 -> CU slot."""
import collections
import sys

rows = [list(map(int, ln.split())) for ln in open(sys.argv[1]) if ln.strip()]
by_cu = collections.defaultdict(list)
xcc_ok = 0
for b, xcc, hw, cu, simd, t0, t1 in rows:
    se = (hw >> 13) & 7
    by_cu[(xcc, se, cu)].append((b, simd))
    xcc_ok += (b % 8) == xcc
print(f"blocks {len(rows)}, block % 8 == xcc for {xcc_ok}")
print(f"distinct CUs {len(by_cu)}; blocks per CU: {collections.Counter(len(v) for v in by_cu.values())}")
t0s = sorted(r[5] for r in rows)
print(f"start spread (100 MHz ticks): {t0s[-1] - t0s[0]}")
for key in sorted(by_cu)[:6]:
    bl = sorted(by_cu[key])
    print(key, [b for b, _ in bl][:20], "simd", [s for _, s in bl][:20])
# (block / 8) residues that share a CU
res = collections.Counter()
for key, bl in by_cu.items():
    slots = sorted({(b // 8) % 32 for b, _ in bl})
    res[len(slots)] += 1
print("distinct (block/8)%32 per CU:", dict(res))
