#!/usr/bin/env python3
"""Generate rot_bench.hip: issue cost on gfx950 of rotate building blocks that
might avoid the half-rate class (v_alignbit_b32 / v_lshlrev_b32 / v_perm_b32):
packed 16-bit shifts and swaps, SDWA sub-dword forms, and whole ChaCha
double-round bodies built from them.  8 waves per SIMD, independent streams.

    python3 tools/ubench/gen_rot_bench.py && hipcc -O3 --offload-arch=gfx950 \
        tools/ubench/rot_bench.hip -o tools/ubench/rot_bench
"""
import os

SINGLE = {
    "add": "v_add_u32 v{d}, v{d}, v{s}",
    "alignbit": "v_alignbit_b32 v{d}, v{d}, v{d}, 20",
    "lshr": "v_lshrrev_b32 v{d}, 3, v{d}",
    "lshl": "v_lshlrev_b32 v{d}, 3, v{d}",
    "perm": "v_perm_b32 v{d}, v{d}, v{d}, v{s}",
    "pk_lshl16": "v_pk_lshlrev_b16 v{d}, 12, v{d}",
    "pk_lshr16_sw": "v_pk_lshrrev_b16 v{d}, 4, v{d} op_sel:[0,1] op_sel_hi:[1,0]",
    "pk_mul16": "v_pk_mul_lo_u16 v{d}, v{d}, v{s}",
    "pk_add16_sw": "v_pk_add_u16 v{d}, v{d}, 0 op_sel:[1,0] op_sel_hi:[0,1]",
    "pk_add16": "v_pk_add_u16 v{d}, v{d}, v{s}",
    "lshl16": "v_lshlrev_b16 v{d}, 3, v{d}",
    "or3": "v_or3_b32 v{d}, v{d}, v{s}, v{d}",
    "lshl_add": "v_lshl_add_u32 v{d}, v{d}, 3, v{s}",
    "xor_sdwa_w": "v_xor_b32_sdwa v{d}, v{d}, v{s} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0",
    "xor_sdwa_dw": "v_xor_b32_sdwa v{d}, v{d}, v{s} dst_sel:DWORD dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD",
    "mov_sdwa_b": "v_mov_b32_sdwa v{d}, v{s} dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0",
    "lshl_sdwa": "v_lshlrev_b32_sdwa v{d}, v{s}, v{d} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_0",
    "mov_dpp": "v_mov_b32_dpp v{d}, v{s} quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
    "bitop3": "v_bitop3_b32 v{d}, v{d}, v{s}, v{d} bitop3:0x96",
    "mad64": "v_mad_u64_u32 v[{d2}:{d3}], vcc, v{d}, v{s}, v[{d2}:{d3}]",
    "mul_u32_u24": "v_mul_u32_u24 v{d}, v{d}, v{s}",
    "mul_hi_u32_u24": "v_mul_hi_u32_u24 v{d}, v{d}, v{s}",
    "mad_u32_u16": "v_mad_u32_u16 v{d}, v{d}, v{s}, v{d}",
    "cvt_pk_u16": "v_cvt_pk_u16_u32 v{d}, v{d}, v{s}",
    "add_co": "v_add_co_u32 v{d}, vcc, v{d}, v{s}",
    "addc": "v_addc_co_u32 v{d}, vcc, v{d}, v{s}, vcc",
    "mul_lo_u32": "v_mul_lo_u32 v{d}, v{d}, v{s}",
    "mul_hi_u32": "v_mul_hi_u32 v{d}, v{d}, v{s}",
    "mad_u32_u24": "v_mad_u32_u24 v{d}, v{d}, v{s}, v{d}",
    "pk_mad_u16": "v_pk_mad_u16 v{d}, v{d}, v{s}, v{d}",
    "dot2_u32_u16": "v_dot2_u32_u16 v{d}, v{d}, v{s}, v{d}",
    "fma_f64": "v_fma_f64 v[{d2}:{d3}], v[{d2}:{d3}], v[{s2}:{s3}], v[{d2}:{d3}]",
    "mul_f64": "v_mul_f64 v[{d2}:{d3}], v[{d2}:{d3}], v[{s2}:{s3}]",
    "pk_fma_f32": "v_pk_fma_f32 v[{d2}:{d3}], v[{d2}:{d3}], v[{s2}:{s3}], v[{d2}:{d3}]",
    "fma_f32": "v_fma_f32 v{d}, v{d}, v{s}, v{d}",
    "cvt_f32_u32": "v_cvt_f32_u32 v{d}, v{d}",
}


def single(fmt, n=64):
    out = []
    for i in range(n):
        d = i % 16
        s = (d + 8) % 16
        d2 = (2 * i) % 16
        out.append(fmt.format(d=d, s=s, d2=d2, d3=d2 + 1, s2=(d2 + 8) % 16, s3=(d2 + 9) % 16))
    return out


A, B, C, D = range(0, 4), range(4, 8), range(8, 12), range(12, 16)
STEPS = [(A, B, D, 16), (C, D, B, 12), (A, B, D, 8), (C, D, B, 7)]
T = 16  # v16..v23: temporaries


def rot_ops(style, z, r, i):
    """Ops rotating v[z] left by r in place (after the xor); temps v16+i, v20+i."""
    t, u = 16 + i, 20 + i
    if style == "alignbit" or (style.startswith("hyb") and r in (12, 7)):
        return ["v_alignbit_b32 v%d, v%d, v%d, %d" % (z, z, z, 32 - r)]
    if r == 16:
        return ["v_pk_add_u16 v%d, v%d, 0 op_sel:[1,0] op_sel_hi:[0,1]" % (z, z)]
    if style == "pkmul":
        return ["v_pk_mul_lo_u16 v%d, v%d, %d" % (t, z, 1 << r) if (1 << r) <= 64 else
                "v_pk_lshlrev_b16 v%d, %d, v%d" % (t, r, z),
                "v_pk_lshrrev_b16 v%d, %d, v%d op_sel:[0,1] op_sel_hi:[1,0]" % (u, 16 - r, z),
                "v_or_b32 v%d, v%d, v%d" % (z, t, u)]
    return ["v_pk_lshlrev_b16 v%d, %d, v%d" % (t, r, z),
            "v_pk_lshrrev_b16 v%d, %d, v%d op_sel:[0,1] op_sel_hi:[1,0]" % (u, 16 - r, z),
            "v_or_b32 v%d, v%d, v%d" % (z, t, u)]


def chacha(style, groups=2):
    out = []
    for _ in range(groups):
        for (x, y, z, r) in STEPS:
            for i in range(4):
                out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
            for i in range(4):
                out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
            rots = [rot_ops(style, z[i], r, i) for i in range(4)]
            for k in range(len(rots[0])):
                for i in range(4):
                    out.append(rots[i][k])
    return out


def chacha_sdwa16(groups=2):
    """xor+rot16 as two SDWA xors writing the swapped halves; other rotations pk16."""
    out = []
    for _ in range(groups):
        for (x, y, z, r) in STEPS:
            for i in range(4):
                out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
            if r == 16:
                for i in range(4):
                    out.append("v_xor_b32_sdwa v%d, v%d, v%d dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE "
                               "src0_sel:WORD_0 src1_sel:WORD_0" % (16 + i, z[i], x[i]))
                for i in range(4):
                    out.append("v_xor_b32_sdwa v%d, v%d, v%d dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE "
                               "src0_sel:WORD_1 src1_sel:WORD_1" % (16 + i, z[i], x[i]))
                for i in range(4):
                    out.append("v_mov_b32 v%d, v%d" % (z[i], 16 + i))  # stand-in for register renaming
                continue
            for i in range(4):
                out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
            rots = [rot_ops("pk", z[i], r, i) for i in range(4)]
            for k in range(len(rots[0])):
                for i in range(4):
                    out.append(rots[i][k])
    return out


def mixed_stream(fast, slow, nf, ns, total=96):
    out = []
    i = 0
    while len(out) < total:
        for _ in range(nf):
            d = i % 16
            out.append(fast.format(d=d, s=(d + 8) % 16))
            i += 1
        for _ in range(ns):
            d = i % 16
            out.append(slow.format(d=d, s=(d + 8) % 16))
            i += 1
    return out[:total]



SINGLE2 = {
    "add": "v_add_u32 v{d}, v{d}, v{s}",
    "alignbit": "v_alignbit_b32 v{d}, v{d}, v{d}, 20",
    "pack_f16": "v_pack_b32_f16 v{d}, v{d}, v{s} op_sel:[1,0,0]",
    "mad_u16": "v_mad_u16 v{d}, v{d}, v{s}, v{d}",
    "mad_u16_hi": "v_mad_u16 v{d}, v{d}, v{s}, v{d} op_sel:[1,0,0,1]",
    "bitop3_b16": "v_bitop3_b16 v{d}, v{d}, v{s}, v{d} bitop3:0x96",
    "bitop3_b16_hi": "v_bitop3_b16 v{d}, v{d}, v{s}, v{d} bitop3:0x96 op_sel:[1,1,1,1]",
    "lshr16": "v_lshrrev_b16 v{d}, 3, v{d}",
    "lshl16": "v_lshlrev_b16 v{d}, 3, v{d}",
    "mul_lo_u16": "v_mul_lo_u16 v{d}, v{d}, v{s}",
    "add_u16": "v_add_u16 v{d}, v{d}, v{s}",
    "and": "v_and_b32 v{d}, v{d}, v{s}",
    "mov": "v_mov_b32 v{d}, v{s}",
    "cndmask": "v_cndmask_b32 v{d}, v{d}, v{s}, vcc",
    "max_u32": "v_max_u32 v{d}, v{d}, v{s}",
    "add_f32": "v_add_f32 v{d}, v{d}, v{s}",
    "mul_f32": "v_mul_f32 v{d}, v{d}, v{s}",
    "ldexp": "v_ldexp_f32 v{d}, v{d}, v{s}",
    "cvt_pkrtz": "v_cvt_pkrtz_f16_f32 v{d}, v{d}, v{s}",
    "lshl_or": "v_lshl_or_b32 v{d}, v{d}, 3, v{s}",
    "and_or": "v_and_or_b32 v{d}, v{d}, v{s}, v{d}",
    "add3": "v_add3_u32 v{d}, v{d}, v{s}, v{d}",
    "xor_e64": "v_xor_b32_e64 v{d}, v{d}, v{s}",
    "add_e64": "v_add_u32_e64 v{d}, v{d}, v{s}",
    "lshr_e64": "v_lshrrev_b32_e64 v{d}, 3, v{d}",
    "bitop3_const": "v_bitop3_b32 v{d}, v{d}, s4, v{d} bitop3:0x96",
    "add_lit": "v_add_u32 v{d}, 0x12345, v{d}",
    "xor_sgpr": "v_xor_b32 v{d}, s4, v{d}",
    "mad_u16_sgpr": "v_mad_u16 v{d}, v{d}, s5, v{s}",
}

def dep_chain(n=64):
    return ["v_add_u32 v0, v0, v1"] * n

def ff(pattern):
    """F/S pattern of independent ops: F = v_add_u32, S = v_alignbit."""
    out = []
    for i, ch in enumerate(pattern):
        d = i % 16; s = (d + 8) % 16
        out.append(("v_add_u32 v%d, v%d, v%d" if ch == "F" else "v_alignbit_b32 v%d, v%d, v%d, 20") % (d, s if ch=="F" else d, d if ch=="S" else d) if ch=="S" else "v_add_u32 v%d, v%d, v%d" % (d, d, s))
    return out

VARIANTS = {"1_" + k: single(v) for k, v in SINGLE2.items()}
VARIANTS["dep_add"] = dep_chain()
VARIANTS["dep2_add"] = ["v_add_u32 v0, v0, v1", "v_add_u32 v2, v2, v3"] * 32
VARIANTS["dep4_add"] = ["v_add_u32 v0, v0, v1", "v_add_u32 v2, v2, v3", "v_add_u32 v4, v4, v5", "v_add_u32 v6, v6, v7"] * 16
for nf, ns in [(8,1),(16,1),(32,1),(64,1),(128,1),(256,1),(4,2),(8,4),(16,8),(32,16),(64,32),(128,64),(256,128),(2,1)]:
    VARIANTS["F%dS%d" % (nf, ns)] = ff(("F" * nf + "S" * ns) * max(1, 96 // (nf + ns)))
VARIANTS["cc_alignbit"] = chacha("alignbit")
HDR = r'''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
'''


def kernel(name, insts):
    body = "\\n\\t".join(insts)
    clob = ",".join('"v%d"' % i for i in range(24))
    return r'''
__global__ void k_%s(uint32_t *out, uint32_t seed) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("%s" ::: %s, "vcc");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = (uint32_t)(t1 - t0); out[2 * blockIdx.x + 1] = (uint32_t)(r1 - r0); }
}
''' % (name, body, clob)


MAIN = r'''
static void run(const char *name, void (*k)(uint32_t *, uint32_t), int ninst, int wps) {
  const int threads = 256, blocks = 256 * wps;
  uint32_t *out; (void)hipMalloc(&out, 8 * blocks + 64);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, 7u);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  double per_simd = 5.0 * blocks * 4 * (double)ITERS * ninst / 1024.0;
  static uint32_t h[65536]; (void)hipMemcpy(h, out, 8 * blocks, hipMemcpyDeviceToHost);
  double clk = 0; for (int b = 0; b < blocks; ++b) clk += (double)h[2 * b] / h[2 * b + 1] * 100.0; clk /= blocks;
  printf("%%-20s ninst=%%3d  %%.2f cyc/inst at %%.0f MHz  (%%.1f cyc per body)\n", name, ninst,
         ms * 1e-3 * clk * 1e6 / per_simd, clk, ms * 1e-3 * clk * 1e6 / per_simd * ninst);
  (void)hipFree(out);
}
int main() {
  for (int w : {8}) {
    printf("== %%d waves per SIMD\n", w);
%s
  }
}
'''

src = HDR
calls = []
for n, ins in VARIANTS.items():
    src += kernel(n, ins)
    calls.append('    run("%s", k_%s, %d, w);' % (n, n, len(ins)))
src += MAIN % "\n".join(calls)
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "mode_bench.hip"), "w").write(src)
