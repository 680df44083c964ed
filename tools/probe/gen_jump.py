"""Generate tools/probe/jump.hip: probe of computed-jump bodies + VGPR index
mode on gfx950 (measurement only).  Variants: (name, vbase, MT, PER, mode)
acc planes v[vbase + 8m + j] (m < MT), x planes v[vbase + 8MT + i];
mode 0 = straight line, 1 = swappc per body, 2 = threaded (body tail jumps
to the next body through an SGPR target table read with s_movrels), 3 = as 1
without VGPR index mode (bodies all hit row 0: timing only)."""
import os
NB = 16
VARIANTS = [("s_v40_mt8_p1", 40, 8, 1, 0), ("j_v40_mt8_p1", 40, 8, 1, 1), ("j_v40_mt8_p2", 40, 8, 2, 1)]


def kernel(name, vb, MT, PER, mode):
    X = vb + 8 * MT
    body = []
    B = body.append
    for i in range(8):
        B(f'v_mov_b32 v{X + i}, %[x{i}]')
    for r in range(vb, vb + 8 * MT):
        B(f'v_mov_b32 v{r}, 0')
    B('s_mov_b32 %[cnt], %[iters]')
    B('s_getpc_b64 s[90:91]')
    B('.Lpc_%=:')
    if mode == 2:   # target table s[20 + 2m : 21 + 2m] for m < MT, then the loop return
        for m in range(MT):
            c = (m * 5 + 3) % NB
            B(f's_add_u32 s{60 + 2 * m}, s90, .Lbody{c}_%= - .Lpc_%=')
            B(f's_addc_u32 s{61 + 2 * m}, s91, 0')
        B(f's_add_u32 s{60 + 2 * MT}, s90, .Lret_%= - .Lpc_%=')
        B(f's_addc_u32 s{61 + 2 * MT}, s91, 0')
    B('.Lloop_%=:')
    if mode == 0:
        for m in range(MT):
            c = (m * 5 + 3) % NB
            for p in range(PER):
                for j in range(8):
                    a = X + (j + c + p) % 8
                    b = X + (j + 3 * c + 2 * p + 1) % 8
                    B(f'v_bitop3_b32 v{vb + 8 * m + j}, v{vb + 8 * m + j}, v{a}, v{b} bitop3:0x96')
    elif mode == 4:   # index mode on for the whole row; bodies advance M0 by 8
        B('s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)')
        for m in range(MT):
            c = (m * 5 + 3) % NB
            B(f's_add_u32 s92, s90, .Lbody{c}_%= - .Lpc_%=')
            B('s_addc_u32 s93, s91, 0')
            B('s_swappc_b64 s[94:95], s[92:93]')
        B('s_set_gpr_idx_off')
    elif mode in (1, 3):
        for m in range(MT):
            c = (m * 5 + 3) % NB
            B(f's_add_u32 s92, s90, .Lbody{c}_%= - .Lpc_%=')
            B('s_addc_u32 s93, s91, 0')
            if mode == 1:
                B(f's_set_gpr_idx_on {8 * m}, gpr_idx(SRC0,DST)')
            B('s_swappc_b64 s[94:95], s[92:93]')
            if mode == 1:
                B('s_set_gpr_idx_off')
    else:
        # M0 = 8m drives both the VGPR index and (divided) the next-target pick
        B('s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)')
        B('s_mov_b64 s[92:93], s[60:61]')
        B('s_setpc_b64 s[92:93]')
        B('.Lret_%=:')
        B('s_set_gpr_idx_off')
    B('s_sub_u32 %[cnt], %[cnt], 1')
    B('s_cmp_lg_u32 %[cnt], 0')
    B('s_cbranch_scc1 .Lloop_%=')
    B('s_branch .Lend_%=')
    for c in range(NB):
        B(f'.Lbody{c}_%=:')
        for p in range(PER):
            for j in range(8):
                a = X + (j + c + p) % 8
                b = X + (j + 3 * c + 2 * p + 1) % 8
                B(f'v_bitop3_b32 v{vb + j}, v{vb + j}, v{a}, v{b} bitop3:0x96')
        if mode == 2:
            # M0 = mode bits | 8m in index mode: entry m+1 of the target table
            # s[60 + 2j] is read with M0 = 2m, then M0 = mode bits | 8(m+1)
            B('s_mov_b32 s96, m0')
            B('s_and_b32 s97, s96, 0xff')
            B('s_lshr_b32 s97, s97, 2')
            B('s_mov_b32 m0, s97')
            B('s_nop 0')
            B('s_movrels_b64 s[92:93], s[62:63]')
            B('s_add_u32 m0, s96, 8')
            B('s_setpc_b64 s[92:93]')
        elif mode == 4:
            B('s_add_u32 m0, m0, 8')
            B('s_setpc_b64 s[94:95]')
        else:
            B('s_setpc_b64 s[94:95]')
    B('.Lend_%=:')
    for r in range(8 * MT):
        B(f'v_mov_b32 %[r{r}], v{vb + r}')
    asm = "\\n\\t".join(body)
    outs = ", ".join(f'[r{r}] "=v"(res[{r}])' for r in range(8 * MT))
    clob_v = ", ".join(f'"v{r}"' for r in range(vb, X + 8))
    clob_s = ", ".join(f'"s{r}"' for r in list(range(60, 62 + 2 * MT)) + list(range(90, 98)))
    ins = ", ".join(f'[x{i}] "v"(xin[{i}])' for i in range(8))
    return f'''
__global__ __launch_bounds__(256) void {name}(uint32_t* out, const uint32_t* in, int iters) {{
  extern __shared__ uint32_t pad[];
  if (iters < 0) pad[threadIdx.x] = 0;
  const int t = blockIdx.x * 256 + threadIdx.x;
  uint32_t xin[8];
  for (int i = 0; i < 8; i++) xin[i] = in[(t * 8 + i) & 4095];
  uint32_t res[{8 * MT}];
  uint32_t cnt;
  asm volatile("{asm}"
      : {outs}, [cnt] "=&s"(cnt)
      : {ins}, [iters] "s"(iters)
      : {clob_v}, {clob_s}, "m0", "scc", "memory");
  if (iters == 1) {{ for (int r = 0; r < {8 * MT}; r++) out[t * 64 + r] = res[r]; }}
  else {{ uint32_t s = 0; for (int r = 0; r < {8 * MT}; r++) s ^= res[r]; out[t] = s; }}
}}
'''


src = ['#include <hip/hip_runtime.h>', '#include <stdint.h>']
for v in VARIANTS:
    src.append(kernel(*v))
src.append('extern "C" int probe_jump(int v, void* out, const void* in, int blocks, int iters, void* stream, int lds) {')
src.append('  hipStream_t st = (hipStream_t)stream;')
for i, v in enumerate(VARIANTS):
    src.append(f'  if (v == {i}) hipLaunchKernelGGL({v[0]}, dim3(blocks), dim3(256), lds, st, (uint32_t*)out, (const uint32_t*)in, iters);')
src.append('  return (int)hipGetLastError();')
src.append('}')
src.append('extern "C" int probe_count() { return %d; }' % len(VARIANTS))
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jump.hip"), "w").write("\n".join(src) + "\n")
