"""Generate tools/probe/dispatch.hip: cost of reaching per-coefficient code
bodies on gfx950 (measurement only, never part of the library).

Every variant computes, per wave and iteration, 8 "rows" m; row m applies
body c_m = (5m + 3) % NB: 8 XOR3s of two input planes into accumulator
planes acc[8m .. 8m+7].  Variants differ only in how the body is reached:

  S  straight line (the VALU floor)
  A  per body: target add/addc, s_set_gpr_idx_on 8m, s_swappc, body,
     s_setpc back, s_set_gpr_idx_off                 (the kernel today)
  B  index mode on for the whole row; targets hoisted; per body s_swappc;
     body tail: s_add_u32 m0, m0, 8 + s_setpc back    (2 redirects, 2 SALU)
  C  threaded copies: one copy of the bodies per m with fixed accumulators;
     body tail s_setpc to the next row's target (hoisted)  (1 redirect)
  D  as C, targets recomputed every iteration (16 SALU per 8 bodies)
  F  as B, but bodies reached with s_setpc and returning through a per-m
     stub table (no swappc)
"""
import os

NB = 16
ACC = 40
X = ACC + 72


def planes(c, j, p=0):
    return X + (j + c + p) % 8, X + (j + 3 * c + 2 * p + 1) % 8


def body_xors(c, accbase):
    out = []
    for j in range(8):
        a, b = planes(c, j)
        out.append(f"v_bitop3_b32 v{accbase + j}, v{accbase + j}, v{a}, v{b} bitop3:0x96")
    return out


def body_xors_hi(c, accbase):
    """The same body on the lane's second block (planes X+8..X+15)."""
    out = []
    for j in range(8):
        a, b = planes(c, j)
        out.append(f"v_bitop3_b32 v{accbase + j}, v{accbase + j}, v{a + 8}, v{b + 8} bitop3:0x96")
    return out


def coef(m, nb=NB, it=None):
    if it is None:
        return (5 * m + 3) % nb
    return ((it * 8 + m) * 29 + 3) % nb


def kernel_bank(name, conflict):
    """Straight-line XOR3s, 8 accumulators x 8 per iteration, operand banks
    (register mod 4) all different (conflict=0) or all equal (conflict=1)."""
    L = []
    B = L.append
    # planes: 16 source registers X..X+15; acc at ACC..ACC+63
    for i in range(8):
        B(f"v_mov_b32 v{X + i}, %[x{i}]")
        B(f"v_mov_b32 v{X + 8 + i}, %[x{i}]")
    for r in range(ACC, ACC + 64):
        B(f"v_mov_b32 v{r}, 0")
    B("s_mov_b32 %[cnt], %[iters]")
    B(".Lloop_%=:")
    for m in range(8):
        for j in range(8):
            a = ACC + 8 * m + j          # bank a % 4
            if conflict:
                srcs = [r for r in range(X, X + 16) if r % 4 == a % 4]
            else:
                srcs = [r for r in range(X, X + 16) if r % 4 not in (a % 4,)]
                srcs = [r for r in srcs if r % 4 == (a + 1) % 4] + [r for r in srcs if r % 4 == (a + 2) % 4]
            s1 = srcs[(m + j) % 2]
            s2 = srcs[2 + (m + j) % 2] if not conflict else srcs[(m + j + 1) % len(srcs)]
            B(f"v_bitop3_b32 v{a}, v{a}, v{s1}, v{s2} bitop3:0x96")
    B("s_sub_u32 %[cnt], %[cnt], 1")
    B("s_cmp_lg_u32 %[cnt], 0")
    B("s_cbranch_scc1 .Lloop_%=")
    for r in range(16):
        B(f"v_bitop3_b32 v{ACC + r}, v{ACC + r}, v{ACC + r + 16}, v{ACC + r + 32} bitop3:0x96")
        B(f"v_xor_b32 %[r{r}], v{ACC + r}, v{ACC + r + 48}")
    asm = "\\n\\t".join(L)
    outs = ", ".join(f'[r{r}] "=v"(res[{r}])' for r in range(16))
    clob_v = ", ".join(f'"v{r}"' for r in range(ACC, X + 16))
    ins = ", ".join(f'[x{i}] "v"(xin[{i}])' for i in range(8))
    return f'''
__global__ __launch_bounds__(256) void {name}(uint32_t* out, const uint32_t* in, int iters) {{
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = 0;
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t xin[8];
  for (int i = 0; i < 8; i++) xin[i] = in[(t * 8 + i) & 4095];
  uint32_t res[16];
  uint32_t cnt;
  asm volatile("{asm}"
      : {outs}, [cnt] "=&s"(cnt)
      : {ins}, [iters] "s"(iters)
      : {clob_v}, "scc", "memory");
  uint32_t s = 0; for (int r = 0; r < 16; r++) s ^= res[r]; out[t] = s;
}}
'''


def kernel(name, mode, nb=NB, dyn=False, ncopy=8):
    L = []
    B = L.append
    wide = mode == "W"
    if wide:
        mode = "T"
    for i in range(8):
        B(f"v_mov_b32 v{X + i}, %[x{i}]")
    if wide:  # second 32-byte block of the lane: the same words rotated by one
        for i in range(8):
            B(f"v_mov_b32 v{X + 8 + i}, %[x{(i + 1) % 8}]")
    for r in range(ACC, ACC + 64):
        B(f"v_mov_b32 v{r}, 0")
    B("s_mov_b32 %[cnt], %[iters]")
    B("s_getpc_b64 s[90:91]")
    B(".Lpc_%=:")
    # hoisted targets s[60+2m : 61+2m]
    if mode in ("B", "F"):
        for m in range(8):
            B(f"s_add_u32 s{60 + 2 * m}, s90, .Lb{coef(m)}_%= - .Lpc_%=")
            B(f"s_addc_u32 s{61 + 2 * m}, s91, 0")
    if mode == "F":
        for m in range(8):
            B(f"s_add_u32 s{34 + 2 * m}, s90, .Lst{m}_%= - .Lpc_%=")
            B(f"s_addc_u32 s{35 + 2 * m}, s91, 0")
    if mode == "C":
        for m in range(8):
            B(f"s_add_u32 s{60 + 2 * m}, s90, .Lc{m}_{coef(m)}_%= - .Lpc_%=")
            B(f"s_addc_u32 s{61 + 2 * m}, s91, 0")
        B("s_add_u32 s76, s90, .Lret_%= - .Lpc_%=")
        B("s_addc_u32 s77, s91, 0")
    if mode == "G" and dyn:
        B("s_add_u32 s98, s90, .Lg0_%= - .Lpc_%=")
        B("s_addc_u32 s99, s91, 0")
    if mode == "D":
        B("s_add_u32 s76, s90, .Lret_%= - .Lpc_%=")
        B("s_addc_u32 s77, s91, 0")
    if mode == "G" and not dyn:
        # slot of row m (read by body m) = target of body m+1; last = return
        for m in range(8):
            if m < 7:
                B(f"s_add_u32 s92, s90, .Lg{coef(m + 1, nb)}_%= - .Lpc_%=")
            else:
                B("s_add_u32 s92, s90, .Lret_%= - .Lpc_%=")
            B(f"v_mov_b32 v{ACC + 9 * m + 8}, s92")
        B(f"s_add_u32 s60, s90, .Lg{coef(0, nb)}_%= - .Lpc_%=")
        B("s_addc_u32 s61, s91, 0")
        B("s_mov_b32 s53, s61")
    if mode == "T":
        R = ncopy
        for m in range(8):
            B(f"s_mov_b32 s{78 + m}, {(5 * m + 3) % nb}")
        for r in range(R):
            B(f"s_add_u32 s{34 + r}, s90, .Lt{r}_0_%= - .Lpc_%=")
    B(".Lloop_%=:")
    if mode == "T":
        R = ncopy
        for ps in range((4 if wide else 8) // R):
            for r in range(R):
                m = ps * R + r
                B(f"s_add_u32 s{78 + m}, s{78 + m}, 232")
                B(f"s_and_b32 s{78 + m}, s{78 + m}, {nb - 1}")
                B(f"s_mul_i32 s92, s{78 + m}, {132 if wide else 68}")  # body bytes: 8 or 16 XOR3 + s_setpc
                B(f"s_add_u32 s{60 + 2 * r}, s92, s{34 + r}")
                B(f"s_addc_u32 s{61 + 2 * r}, s91, 0")
            B(f"s_add_u32 s{60 + 2 * R}, s90, .Lret{ps}_%= - .Lpc_%=")
            B(f"s_addc_u32 s{61 + 2 * R}, s91, 0")
            B("s_setpc_b64 s[60:61]")
            B(f".Lret{ps}_%=:")
    elif mode == "G":
        if dyn:
            # c_m = ((cnt*8 + m)*29 + 3) % nb, bodies GSIZE bytes apart
            for m in range(8):
                B(f"s_lshl_b32 s92, %[cnt], 3")
                B(f"s_add_u32 s92, s92, {m}")
                B("s_mul_i32 s92, s92, 29")
                B("s_add_u32 s92, s92, 3")
                B(f"s_and_b32 s92, s92, {nb - 1}")
                B(f"s_mul_i32 s92, s92, {GSIZE}")
                B(f"s_add_u32 s92, s92, s98")
                if m == 0:
                    B("s_mov_b32 s60, s92")
                else:
                    B(f"v_mov_b32 v{ACC + 9 * (m - 1) + 8}, s92")
            B("s_add_u32 s92, s90, .Lret_%= - .Lpc_%=")
            B(f"v_mov_b32 v{ACC + 9 * 7 + 8}, s92")
            B("s_mov_b32 s61, s99")
            B("s_mov_b32 s53, s99")
        B("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        B("s_setpc_b64 s[60:61]")
        B(".Lret_%=:")
        B("s_set_gpr_idx_off")
    elif mode == "S":
        for m in range(8):
            L.extend(body_xors(coef(m), ACC + 8 * m))
    elif mode == "A":
        for m in range(8):
            B(f"s_add_u32 s92, s90, .Lb{coef(m)}_%= - .Lpc_%=")
            B("s_addc_u32 s93, s91, 0")
            B(f"s_set_gpr_idx_on {8 * m}, gpr_idx(SRC0,DST)")
            B("s_swappc_b64 s[94:95], s[92:93]")
            B("s_set_gpr_idx_off")
    elif mode == "B":
        B("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        for m in range(8):
            B(f"s_swappc_b64 s[94:95], s[{60 + 2 * m}:{61 + 2 * m}]")
        B("s_set_gpr_idx_off")
    elif mode == "F":
        B("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
        B("s_mov_b64 s[94:95], s[34:35]")
        B("s_setpc_b64 s[60:61]")
        for m in range(8):
            B(f".Lst{m}_%=:")
            if m < 7:
                B(f"s_mov_b64 s[94:95], s[{36 + 2 * m}:{37 + 2 * m}]")
                B(f"s_setpc_b64 s[{62 + 2 * m}:{63 + 2 * m}]")
        B("s_set_gpr_idx_off")
    elif mode in ("C", "D"):
        if mode == "D":
            for m in range(8):
                B(f"s_add_u32 s{60 + 2 * m}, s90, .Lc{m}_{coef(m)}_%= - .Lpc_%=")
                B(f"s_addc_u32 s{61 + 2 * m}, s91, 0")
        B("s_setpc_b64 s[60:61]")
        B(".Lret_%=:")
    B("s_sub_u32 %[cnt], %[cnt], 1")
    B("s_cmp_lg_u32 %[cnt], 0")
    B("s_cbranch_scc1 .Lloop_%=")
    B("s_add_u32 s92, s90, .Lend_%= - .Lpc_%=")
    B("s_addc_u32 s93, s91, 0")
    B("s_setpc_b64 s[92:93]")
    if mode in ("A", "B", "F"):
        for c in range(NB):
            B(f".Lb{c}_%=:")
            L.extend(body_xors(c, ACC))
            if mode == "B":
                B("s_add_u32 m0, m0, 8")
            if mode == "F":
                B("s_add_u32 m0, m0, 8")
            B("s_setpc_b64 s[94:95]")
    elif mode in ("C", "D"):
        for m in range(8):
            for c in range(NB):
                B(f".Lc{m}_{c}_%=:")
                L.extend(body_xors(c, ACC + 8 * m))
                B(f"s_setpc_b64 s[{62 + 2 * m}:{63 + 2 * m}]")
    if mode == "T":
        for r in range(ncopy):
            for c in range(nb):
                B(f".Lt{r}_{c}_%=:")
                if wide:
                    L.extend(body_xors(c, ACC + 16 * r))
                    L.extend(body_xors_hi(c, ACC + 16 * r + 8))
                else:
                    L.extend(body_xors(c, ACC + 8 * r))
                B(f"s_setpc_b64 s[{62 + 2 * r}:{63 + 2 * r}]")
    if mode == "G":
        for c in range(nb):
            B(f".Lg{c}_%=:")
            B(f"v_readfirstlane_b32 s52, v{ACC + 8}")
            L.extend(body_xors(c, ACC))
            B("s_add_u32 m0, m0, 9")
            B("s_setpc_b64 s[52:53]")
    B(".Lend_%=:")
    if mode == "G":   # back to stride 8 for the fold
        for m in range(1, 8):
            for j in range(8):
                B(f"v_mov_b32 v{ACC + 8 * m + j}, v{ACC + 9 * m + j}")
    # fold the 64 accumulators to 16 outputs: r ^ r+16 ^ r+32 ^ r+48
    for r in range(16):
        B(f"v_bitop3_b32 v{ACC + r}, v{ACC + r}, v{ACC + r + 16}, v{ACC + r + 32} bitop3:0x96")
        B(f"v_xor_b32 %[r{r}], v{ACC + r}, v{ACC + r + 48}")
    asm = "\\n\\t".join(L)
    outs = ", ".join(f'[r{r}] "=v"(res[{r}])' for r in range(16))
    clob_v = ", ".join(f'"v{r}"' for r in range(ACC, X + (16 if wide else 8)))
    clob_s = ", ".join(f'"s{r}"' for r in list(range(34, 50)) + list(range(60, 88)) + list(range(90, 100)))
    ins = ", ".join(f'[x{i}] "v"(xin[{i}])' for i in range(8))
    return f'''
__global__ __launch_bounds__(256) void {name}(uint32_t* out, const uint32_t* in, int iters) {{
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = 0;
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t xin[8];
  for (int i = 0; i < 8; i++) xin[i] = in[(t * 8 + i) & 4095];
  uint32_t res[16];
  uint32_t cnt;
  asm volatile("{asm}"
      : {outs}, [cnt] "=&s"(cnt)
      : {ins}, [iters] "s"(iters)
      : {clob_v}, {clob_s}, "m0", "scc", "memory");
  if (iters == 1) {{ for (int r = 0; r < 16; r++) out[t * 16 + r] = res[r]; }}
  else {{ uint32_t s = 0; for (int r = 0; r < 16; r++) s ^= res[r]; out[t] = s; }}
}}
'''


GSIZE = 4 + 64 + 4 + 4
VARIANTS = [("S", "S", NB, False), ("A", "A", NB, False), ("B", "B", NB, False), ("C", "C", NB, False),
            ("D", "D", NB, False), ("T16r8", "T", 16, True, 8), ("T256r8", "T", 256, True, 8),
            ("T256r4", "T", 256, True, 4), ("T16r4", "T", 16, True, 4), ("T128r8", "T", 128, True, 8),
            ("T64r8", "T", 64, True, 8), ("bank_ok", "BANK", 0, False), ("bank_conflict", "BANK", 1, False),
            ("W256r4", "W", 256, True, 4), ("W16r4", "W", 16, True, 4)]


def main():
    src = ["#include <hip/hip_runtime.h>", "#include <stdint.h>"]
    for v in VARIANTS:
        if v[1] == "BANK":
            src.append(kernel_bank(f"disp_{v[0]}", v[2]))
        else:
            src.append(kernel(f"disp_{v[0]}", *v[1:]))
    src.append('extern "C" int probe_dispatch(int v, void* out, const void* in, int blocks, int iters, '
               'void* stream, int lds) {')
    src.append("  hipStream_t st = (hipStream_t)stream;")
    for i, v in enumerate(VARIANTS):
        src.append(f"  if (v == {i}) hipLaunchKernelGGL(disp_{v[0]}, dim3(blocks), dim3(256), lds, st, "
                   "(uint32_t*)out, (const uint32_t*)in, iters);")
    src.append("  return (int)hipGetLastError();")
    src.append("}")
    here = os.path.dirname(os.path.abspath(__file__))
    open(os.path.join(here, "dispatch.hip"), "w").write("\n".join(src) + "\n")


if __name__ == "__main__":
    main()
