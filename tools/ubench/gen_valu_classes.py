#!/usr/bin/env python3
"""Generate valu_classes.hip: round-2 probe of gfx950 VALU issue classes for
the instructions an all-"fast"-class ChaCha20 rotation could use (24-bit
multiplies, 16-bit multiplies, bitop3, literal / SGPR operands), and whole
ChaCha quarter-round groups written three ways, at 8 and 2 waves per SIMD.

Background (profiles/round1, tools/ubench/gen_issue_bench.py): on gfx950
v_add/v_xor/v_lshrrev issue at ~2 cycles per wave64 instruction when several
waves interleave, v_alignbit at ~4, and a stream mixing the two runs every
instruction at ~4.  A rotation built only from fast-class instructions would
let a ChaCha stream run at ~2 cycles per instruction:
    rotl(x, n), n >= 8:  v_mad_u32_u24(x, 2^n, x >> (32-n))
        (x << n mod 2^32 only needs the low 32-n <= 24 bits of x; the two
        terms have disjoint bits, so + == |)
    rotl(x, 7):  (x[9..24] << 16 via mad24 of x >> 9) | x >> 25 | x[0..8] << 7
        (the last term from v_mul_lo_u16(x, 128): low 16 bits, high zeroed)
"""
import sys

SINGLE = {
    "add": "v_add_u32 v{d}, v{d}, v{s}",
    "alignbit": "v_alignbit_b32 v{d}, v{d}, v{d}, 20",
    "mad24_v": "v_mad_u32_u24 v{d}, v{d}, v20, v{s}",
    "mad24_i": "v_mad_u32_u24 v{d}, v{d}, 64, v{s}",
    "mad24_s": "v_mad_u32_u24 v{d}, v{d}, s20, v{s}",
    "mul24_v": "v_mul_u32_u24 v{d}, v{d}, v20",
    "mul24_i": "v_mul_u32_u24 v{d}, 64, v{d}",
    "mulhi24": "v_mul_hi_u32_u24 v{d}, v{d}, v20",
    "mul_lo_u16_i": "v_mul_lo_u16 v{d}, 64, v{d}",
    "mul_lo_u16_v": "v_mul_lo_u16 v{d}, v20, v{d}",
    "bitop3_3v": "v_bitop3_b32 v{d}, v{d}, v{s}, v{t} bitop3:0xfe",
    "and_lit": "v_and_b32 v{d}, 0xff, v{d}",
    "xor_s": "v_xor_b32 v{d}, s20, v{d}",
    "add_s": "v_add_u32 v{d}, s20, v{d}",
    "perm": "v_perm_b32 v{d}, v{d}, v{d}, v20",
    "add3": "v_add3_u32 v{d}, v{d}, v{s}, v{t}",
    "lshl_add": "v_lshl_add_u32 v{d}, v{d}, 3, v{s}",
    "lshl_vv": "v_lshlrev_b32 v{d}, v21, v{d}",
    "mul_lo_u32": "v_mul_lo_u32 v{d}, v{d}, v{s}",
    "lshr_b16": "v_lshrrev_b16 v{d}, 3, v{d}",
    "sub_rev": "v_subrev_u32 v{d}, v{d}, v{s}",
    "not": "v_not_b32 v{d}, v{d}",
    "mad_u32_u16": "v_mad_u32_u16 v{d}, v{d}, v20, v{s}",
    "lshr_vv": "v_lshrrev_b32 v{d}, v21, v{d}",
    "mov_s": "v_mov_b32 v{d}, s20",
    "cnd_vcc": "v_cndmask_b32_e32 v{d}, v{d}, v{s}, vcc",
    "cnd_sgpr": "v_cndmask_b32_e64 v{d}, v{d}, v{s}, s[20:21]",
    "addc": "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc",
}


def pairs(fmt_list, n=64):
    """repeat a short dependent sequence (e.g. an add-with-carry chain)"""
    out = []
    for i in range(n // len(fmt_list)):
        d = (i * len(fmt_list)) % 16
        for k, f in enumerate(fmt_list):
            e = (2 * (d + k)) % 16
            out.append(f.format(d=(d + k) % 16, s=(d + k + 8) % 16, t=(d + k + 4) % 16, d2=e, d3=e + 1))
    return out


CHAINS = {
    # h + m with full carry propagation, then the carry materialised (poly_block as compiled)
    "chain_add5_cnd": ["v_add_co_u32_e32 v{d}, vcc, v{d}, v{s}", "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc",
                       "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc", "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc",
                       "v_cndmask_b32_e64 v{t}, 0, 1, vcc"],
    "chain_add5_addc": ["v_add_co_u32_e32 v{d}, vcc, v{d}, v{s}", "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc",
                        "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc", "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc",
                        "v_addc_co_u32_e32 v{t}, vcc, 1, v{t}, vcc"],
    "xor_addc_mix": ["v_xor_b32_e32 v{t}, v{t}, v{s}", "v_addc_co_u32_e32 v{d}, vcc, v{d}, v{s}, vcc"],
    "cnd_e64_vcc": ["v_cndmask_b32_e64 v{d}, v{d}, v{s}, vcc"],
    "cmp_cnd_vcc": ["v_cmp_gt_u32_e32 vcc, v{d}, v{s}", "v_cndmask_b32_e64 v{t}, 0, 1, vcc"],
    "cmp_cnd_sgpr": ["v_cmp_gt_u32_e64 s[20:21], v{d}, v{s}", "v_cndmask_b32_e64 v{t}, 0, 1, s[20:21]"],
    "cmp_cnd_sgpr2": ["v_cmp_gt_u32_e64 s[20:21], v{d}, v{s}", "v_cmp_gt_u32_e64 s[22:23], v{s}, v{d}",
                      "v_cndmask_b32_e64 v{t}, 0, 1, s[20:21]", "v_cndmask_b32_e64 v{d}, 0, 1, s[22:23]"],
    "mad64_vcc": ["v_mad_u64_u32 v[16:17], vcc, v{d}, v{s}, v[16:17]"],
    "mad64_sdst": ["v_mad_u64_u32 v[16:17], s[20:21], v{d}, v{s}, v[16:17]"],
    "mad64_4acc_sdst": ["v_mad_u64_u32 v[16:17], s[20:21], v{d}, v{s}, v[16:17]",
                        "v_mad_u64_u32 v[18:19], s[20:21], v{d}, v{t}, v[18:19]",
                        "v_mad_u64_u32 v[24:25], s[20:21], v{s}, v{t}, v[24:25]",
                        "v_mad_u64_u32 v[26:27], s[20:21], v{t}, v{d}, v[26:27]"],
    "mad64_4acc_rot": ["v_mad_u64_u32 v[16:17], s[20:21], v{d}, v{s}, v[16:17]",
                       "v_mad_u64_u32 v[18:19], s[22:23], v{d}, v{t}, v[18:19]",
                       "v_mad_u64_u32 v[24:25], s[24:25], v{s}, v{t}, v[24:25]",
                       "v_mad_u64_u32 v[26:27], s[26:27], v{t}, v{d}, v[26:27]"],
    "xor_mad_mix": ["v_xor_b32_e32 v{t}, v{t}, v{s}", "v_mad_u64_u32 v[16:17], s[20:21], v{d}, v{s}, v[16:17]",
                    "v_xor_b32_e32 v{d}, v{d}, v{s}", "v_mad_u64_u32 v[18:19], s[22:23], v{d}, v{t}, v[18:19]"],
    "addc_4chains": ["v_add_co_u32_e64 v{d}, s[20:21], v{d}, v{s}", "v_add_co_u32_e64 v{t}, s[22:23], v{t}, v{s}",
                     "v_add_co_u32_e64 v{s}, s[24:25], v{s}, v{d}", "v_add_co_u32_e64 v28, s[26:27], v28, v{d}",
                     "v_addc_co_u32_e64 v{d}, s[20:21], v{d}, v{s}, s[20:21]",
                     "v_addc_co_u32_e64 v{t}, s[22:23], v{t}, v{s}, s[22:23]",
                     "v_addc_co_u32_e64 v{s}, s[24:25], v{s}, v{d}, s[24:25]",
                     "v_addc_co_u32_e64 v28, s[26:27], v28, v{d}, s[26:27]"],
    "lshl_add64": ["v_lshl_add_u64 v[16:17], v[{d2}:{d3}], 0, v[16:17]"],
}


def single(fmt, n=64):
    out = []
    for i in range(n):
        d = i % 16
        out.append(fmt.format(d=d, s=(d + 8) % 16, t=(d + 4) % 16))
    return out


A, B, C, D = range(0, 4), range(4, 8), range(8, 12), range(12, 16)
STEPS = [(A, B, D, 16), (C, D, B, 12), (A, B, D, 8), (C, D, B, 7)]
# constant registers: v20 = 65536, v21 = 4096, v22 = 256, v23 = 128 (set before the loop)
KREG = {16: 20, 12: 21, 8: 22}


def qr_alignbit(groups=2):
    out = []
    for _ in range(groups):
        for (x, y, z, r) in STEPS:
            for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
            for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
            for i in range(4): out.append("v_alignbit_b32 v%d, v%d, v%d, %d" % (z[i], z[i], z[i], 32 - r))
    return out


def qr_mad24(groups=2, rot7="fast"):
    """all-fast rotations; temps v24..v31"""
    out = []
    for _ in range(groups):
        for (x, y, z, r) in STEPS:
            for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
            for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (z[i], z[i], x[i]))
            if r != 7:
                for i in range(4): out.append("v_lshrrev_b32 v%d, %d, v%d" % (24 + i, 32 - r, z[i]))
                for i in range(4): out.append("v_mad_u32_u24 v%d, v%d, v%d, v%d" % (z[i], z[i], KREG[r], 24 + i))
            elif rot7 == "alignbit":
                for i in range(4): out.append("v_alignbit_b32 v%d, v%d, v%d, 25" % (z[i], z[i], z[i]))
            else:
                # t = x >> 9; u = x >> 25; w = mul_lo_u16(x, 128); x = mad24(t, 65536, u | w)
                for i in range(4): out.append("v_lshrrev_b32 v%d, 9, v%d" % (24 + i, z[i]))
                for i in range(4): out.append("v_lshrrev_b32 v%d, 25, v%d" % (28 + i, z[i]))
                for i in range(4): out.append("v_mul_lo_u16 v%d, v23, v%d" % (z[i], z[i]))
                for i in range(4): out.append("v_or_b32 v%d, v%d, v%d" % (z[i], z[i], 28 + i))
                for i in range(4): out.append("v_mad_u32_u24 v%d, v%d, v20, v%d" % (z[i], 24 + i, z[i]))
    return out


VARIANTS = {"qr_alignbit": qr_alignbit(), "qr_mad24": qr_mad24(), "qr_mad24_r7ab": qr_mad24(rot7="alignbit")}
for k, v in SINGLE.items():
    VARIANTS["1_" + k] = single(v)
for k, v in CHAINS.items():
    VARIANTS[k] = pairs(v, 60)

HDR = r'''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
'''
CLOB = ",".join('"v%d"' % i for i in range(32)) + ',"s20","s21","s22","s23","s24","s25","s26","s27","vcc"'
SETUP = ("v_mov_b32 v20, 0x10000\\n\\tv_mov_b32 v21, 0x1000\\n\\tv_mov_b32 v22, 0x100\\n\\t"
         "v_mov_b32 v23, 0x80\\n\\ts_mov_b32 s20, 0x10000\\n\\ts_mov_b32 s21, 0")


def kernel(name, insts):
    body = "\\n\\t".join(insts)
    return r'''
__global__ void k_%s(uint32_t *out, uint32_t seed) {
  asm volatile("%s" ::: %s);
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("%s" ::: %s);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = (uint32_t)(t1 - t0); out[2 * blockIdx.x + 1] = (uint32_t)(r1 - r0); }
}
''' % (name, SETUP, CLOB, body, CLOB)


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
  printf("%%-16s w/SIMD=%%d  clock %%4.0f MHz  %%.2f cyc/inst\n", name, wps, clk, ms * 1e-3 * clk * 1e6 / per_simd);
  (void)hipFree(out);
}
int main() {
  for (int w : {8, 2}) {
%s
  }
}
'''


def main(path):
    src = HDR
    calls = []
    for n, ins in VARIANTS.items():
        src += kernel(n, ins)
        calls.append('    run("%s", k_%s, %d, w);' % (n, n, len(ins)))
    src += MAIN % "\n".join(calls)
    open(path, "w").write(src)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "valu_classes.hip")
