#!/usr/bin/env python3
"""Generate issue_bench.hip: VALU issue-cost model of gfx950 for instruction
mixes (fast add/xor vs half-rate alignbit/mad64), independent streams and
ChaCha-shaped dependency patterns, at 2 and 8 waves per SIMD."""
F_ADD = "v_add_u32 v{d}, v{d}, v{s}"
F_XOR = "v_xor_b32 v{d}, v{d}, v{s}"
S_ROT = "v_alignbit_b32 v{d}, v{d}, v{d}, 20"

def stream(pattern, nreg=16):
    """pattern: string of F/X/S; each op on its own register (round-robin),
    sources from a register 8 away -> no short dependencies."""
    out = []
    for i, ch in enumerate(pattern):
        d = i % nreg
        s = (d + 8) % nreg
        out.append({"F": F_ADD, "X": F_XOR, "S": S_ROT}[ch].format(d=d, s=s))
    return out

def chacha_like(n_qr_groups=2, style="compiler"):
    """4 parallel QRs (columns) x 12 ops each in the order the compiler emits
    (4 add, 4 xor, 4 rot, ...) over registers v0..v15 (a=0-3, b=4-7, c=8-11, d=12-15)."""
    out = []
    A, B, C, D = range(0, 4), range(4, 8), range(8, 12), range(12, 16)
    steps = [(A, B, D, 16), (C, D, B, 12), (A, B, D, 8), (C, D, B, 7)]
    for _ in range(n_qr_groups):
        for (x, y, z, r) in steps:
            if style == "compiler":
                for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
                for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
                for i in range(4): out.append("v_alignbit_b32 v%d, v%d, v%d, %d" % (z[i], z[i], z[i], 32 - r))
            else:  # per-column chains interleaved one op at a time
                for i in range(4):
                    out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
                    out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
                    out.append("v_alignbit_b32 v%d, v%d, v%d, %d" % (z[i], z[i], z[i], 32 - r))
    return out

SINGLE = {
    "and": "v_and_b32 v{d}, v{d}, v{s}",
    "or": "v_or_b32 v{d}, v{d}, v{s}",
    "sub": "v_sub_u32 v{d}, v{d}, v{s}",
    "mov": "v_mov_b32 v{d}, v{s}",
    "cndmask": "v_cndmask_b32 v{d}, v{d}, v{s}, vcc",
    "bfi": "v_bfi_b32 v{d}, v{d}, v{s}, v{d}",
    "bitop3": "v_bitop3_b32 v{d}, v{d}, v{s}, v{d} bitop3:0x96",
    "lshl_or": "v_lshl_or_b32 v{d}, v{d}, 3, v{s}",
    "alignbyte": "v_alignbyte_b32 v{d}, v{d}, v{d}, 2",
    "bfe": "v_bfe_u32 v{d}, v{d}, 3, 7",
    "pk_add_u16": "v_pk_add_u16 v{d}, v{d}, v{s} op_sel:[1,0] op_sel_hi:[0,1]",
    "pk_lshl_b16": "v_pk_lshlrev_b16 v{d}, 3, v{d}",
    "lshl_b16": "v_lshlrev_b16 v{d}, 3, v{d}",
    "pk_add_f32": "v_pk_add_f32 v[{d2}:{d3}], v[{d2}:{d3}], v[{s2}:{s3}]",
    "fma_f32": "v_fma_f32 v{d}, v{d}, v{s}, v{d}",
    "add_f32": "v_add_f32 v{d}, v{d}, v{s}",
    "mul_f32": "v_mul_f32 v{d}, v{d}, v{s}",
    "xad": "v_xad_u32 v{d}, v{d}, v{s}, v{d}",
    "lshr": "v_lshrrev_b32 v{d}, 3, v{d}",
    "ashr": "v_ashrrev_i32 v{d}, 3, v{d}",
    "add_co": "v_add_co_u32 v{d}, vcc, v{d}, v{s}",
    "mad64": "v_mad_u64_u32 v[{d2}:{d3}], vcc, v{d}, v{s}, v[{d2}:{d3}]",
}
def single(fmt, n=64):
    out = []
    for i in range(n):
        d = i % 16; s = (d + 8) % 16
        d2 = (2 * i) % 16; d3 = d2 + 1; s2 = (d2 + 8) % 16; s3 = s2 + 1
        out.append(fmt.format(d=d, s=s, d2=d2, d3=d3, s2=s2, s3=s3))
    return out

def chacha_fast(n_qr_groups=2):
    """all-fast rotation: t = x ^ y; x = (t << n) | (t >> (32 - n)); uses v16-v19 as temps."""
    out = []
    A, B, C, D = range(0, 4), range(4, 8), range(8, 12), range(12, 16)
    steps = [(A, B, D, 16), (C, D, B, 12), (A, B, D, 8), (C, D, B, 7)]
    for _ in range(n_qr_groups):
        for (x, y, z, r) in steps:
            for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
            for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
            for i in range(4): out.append("v_lshlrev_b32 v%d, %d, v%d" % (16 + i, r, z[i]))
            for i in range(4): out.append("v_lshrrev_b32 v%d, %d, v%d" % (z[i], 32 - r, z[i]))
            for i in range(4): out.append("v_or_b32 v%d, v%d, v%d" % (z[i], z[i], 16 + i))
    return out

def chacha_hybrid(n_qr_groups=2):
    """rot16 and rot8 by v_perm (slow), rot12/rot7 all-fast."""
    out = []
    A, B, C, D = range(0, 4), range(4, 8), range(8, 12), range(12, 16)
    steps = [(A, B, D, 16), (C, D, B, 12), (A, B, D, 8), (C, D, B, 7)]
    for _ in range(n_qr_groups):
        for (x, y, z, r) in steps:
            for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
            for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
            if r in (16, 8):
                for i in range(4): out.append("v_alignbit_b32 v%d, v%d, v%d, %d" % (z[i], z[i], z[i], 32 - r))
            else:
                for i in range(4): out.append("v_lshlrev_b32 v%d, %d, v%d" % (16 + i, r, z[i]))
                for i in range(4): out.append("v_lshrrev_b32 v%d, %d, v%d" % (z[i], 32 - r, z[i]))
                for i in range(4): out.append("v_or_b32 v%d, v%d, v%d" % (z[i], z[i], 16 + i))
    return out

def stream_sep(pattern):
    """F ops on v0-v7, S ops on v8-v15: no register shared between classes."""
    out = []; fi = si = 0
    for ch in pattern:
        if ch == "F":
            d = fi % 8; out.append("v_add_u32 v%d, v%d, v%d" % (d, d, (d + 4) % 8)); fi += 1
        else:
            d = 8 + si % 8; out.append("v_alignbit_b32 v%d, v%d, v%d, 20" % (d, d, d)); si += 1
    return out

VARIANTS = {
    "chacha_ref": chacha_like(2, "compiler"),
    "F16S8": stream(("F" * 16 + "S" * 8) * 4),
    "F32S16": stream(("F" * 32 + "S" * 16) * 2),
    "F64S32": stream("F" * 64 + "S" * 32),
    "F128S64": stream("F" * 128 + "S" * 64),
    "F256S128": stream("F" * 256 + "S" * 128),
    "F255S1": stream("F" * 255 + "S"),
    "F63S1": stream("F" * 63 + "S"),
    "1_lshr64": single("v_lshrrev_b64 v[{d2}:{d3}], 20, v[{d2}:{d3}]"),
    "1_ashr64": single("v_ashrrev_i64 v[{d2}:{d3}], 20, v[{d2}:{d3}]"),
    "1_mov64": single("v_mov_b64 v[{d2}:{d3}], v[{s2}:{s3}]"),
    "1_pk_mov": single("v_pk_mov_b32 v[{d2}:{d3}], v[{d2}:{d3}], v[{s2}:{s3}] op_sel:[1,0]"),
    "1_mul_u16": single("v_mul_lo_u16 v{d}, v{d}, v{s}"),
    "1_lshr_vv": single("v_lshrrev_b32 v{d}, v{s}, v{d}"),
    "1_add_u16": single("v_add_u16 v{d}, v{d}, v{s}"),
    "1_cvt": single("v_cvt_f32_u32 v{d}, v{d}"),
    "F15S1": stream("FFFFFFFFFFFFFFFS" * 4),
    "F7S1": stream("FFFFFFFS" * 8),
    "F1S15": stream("FSSSSSSSSSSSSSSS" * 4),
    "sep_FS": stream_sep("FS" * 32),
    "sep_F3S1": stream_sep("FFFS" * 16),
    "sep_F15S1": stream_sep("FFFFFFFFFFFFFFFS" * 4),
    "chacha_fast": chacha_fast(2),
    "chacha_hybrid": chacha_hybrid(2),
    "1_lshl": single("v_lshlrev_b32 v{d}, 3, v{d}"),
    "F64": stream("F" * 64),
    "X64": stream("X" * 64),
    "S64": stream("S" * 64),
    "FS_alt": stream("FS" * 32),
    "FFS": stream("FFS" * 21),
    "FFFS": stream("FFFS" * 16),
    "FFFFSSSS": stream("FFFFFFFFSSSS" * 5),
    "chacha_cmp": chacha_like(2, "compiler"),
    "chacha_chain": chacha_like(2, "chain"),
}
for k, v in SINGLE.items():
    VARIANTS["1_" + k] = single(v)


HDR = r'''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
'''
def kernel(name, insts):
    body = "\\n\\t".join(insts)
    clob = ",".join('"v%d"' % i for i in range(20))
    return r'''
__global__ void k_%s(uint32_t *out, uint32_t seed) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("%s" ::: %s);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = (uint32_t)(t1 - t0); out[2 * blockIdx.x + 1] = (uint32_t)(r1 - r0); }
}
''' % (name, body, clob)

SPLIT = r'''
__global__ void k_split(uint32_t *out, uint32_t seed) {
  if ((threadIdx.x / 64) & 1) {
    for (int i = 0; i < ITERS; ++i) asm volatile("%s" ::: %s);
  } else {
    for (int i = 0; i < ITERS; ++i) asm volatile("%s" ::: %s);
  }
  if (seed == 12345) out[threadIdx.x] = 0;
}
'''
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
  printf("%%-14s w/SIMD=%%d  %%.2f cyc/inst (@2.2GHz)  in-kernel clock %%.0f MHz -> %%.2f cyc/inst at that clock\n", name, wps, ms * 1e-3 * 2.2e9 / per_simd, clk, ms * 1e-3 * clk * 1e6 / per_simd);
  (void)hipFree(out);
}
int main() {
  for (int w : {8}) {
%s
  }
}
'''
src = HDR
calls = []
for n, ins in VARIANTS.items():
    src += kernel(n, ins)
    calls.append('    run("%s", k_%s, %d, w);' % (n, n, len(ins)))
clob = ",".join('"v%d"' % i for i in range(16))
clob = ",".join('"v%d"' % i for i in range(20))
def addsplit(name, odd, even, n_total_per_pair):
    global src
    ident = name.replace("|", "_")
    src += SPLIT.replace("k_split", "k_" + ident) % ("\\n\\t".join(odd), clob, "\\n\\t".join(even), clob)
    calls.append('    run("%s", k_%s, %d, w);' % (name, ident, n_total_per_pair))
addsplit("split_F|S", stream("S" * 64), stream("F" * 64), 64)
cc = chacha_like(2, "compiler")  # 96 instructions
addsplit("split_cc|cc", cc, cc, 96)
s96 = stream("S" * 96); f96 = stream("F" * 96)
addsplit("split_cc|S", s96, cc, 96)
addsplit("split_cc|F", f96, cc, 96)
src += MAIN % "\n".join(calls)
open("issue_bench.hip", "w").write(src)
