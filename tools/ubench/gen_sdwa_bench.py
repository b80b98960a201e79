#!/usr/bin/env python3
"""Generate sdwa_bench.hip: issue cost of gfx950 SDWA (sub-dword) VOP2 forms,
and a ChaCha quarter-round stream whose xor + rotl 16 pairs are written as
two SDWA xors (high half <- low halves, low half <- high halves) instead of
v_xor + v_alignbit.  Same harness and register layout as gen_valu_classes.py.

Question: is an SDWA xor a fast-class (~2 cycle) instruction, and does a
stream with 3 instead of 4 alignbits per quarter-round issue faster?
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_valu_classes as g  # noqa: E402

SINGLE = {
    "xor_sdwa_w1": "v_xor_b32_sdwa v{d}, v{d}, v{s} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE "
                   "src0_sel:WORD_0 src1_sel:WORD_0",
    "xor_sdwa_pad": "v_xor_b32_sdwa v{d}, v{d}, v{s} dst_sel:WORD_1 dst_unused:UNUSED_PAD "
                    "src0_sel:WORD_0 src1_sel:WORD_0",
    "mov_sdwa": "v_mov_b32_sdwa v{d}, v{s} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0",
    "add_sdwa": "v_add_u32_sdwa v{d}, v{d}, v{s} dst_sel:DWORD dst_unused:UNUSED_PAD "
                "src0_sel:DWORD src1_sel:WORD_1",
    "xor": "v_xor_b32 v{d}, v{d}, v{s}",
    "alignbit": "v_alignbit_b32 v{d}, v{d}, v{d}, 20",
}

A, B, C, D = range(0, 4), range(4, 8), range(8, 12), range(12, 16)
T = range(24, 28)


def qr(groups=2, sdwa16=True):
    """4 parallel quarter-rounds; rotl 16 as two SDWA xors into a spare
    register set (the d registers alternate between v12-15 and v24-27)"""
    out = []
    d = list(D)
    spare = list(T)
    for _ in range(groups):
        for step in range(4):
            if step in (0, 2):   # a += b; d = rotl(d ^ a, 16 / 8)
                x, y, r = A, B, 16 if step == 0 else 8
                for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (x[i], x[i], y[i]))
                if r == 16 and sdwa16:
                    for i in range(4):
                        out.append("v_xor_b32_sdwa v%d, v%d, v%d dst_sel:WORD_1 dst_unused:UNUSED_PAD "
                                   "src0_sel:WORD_0 src1_sel:WORD_0" % (spare[i], d[i], x[i]))
                    for i in range(4):
                        out.append("v_xor_b32_sdwa v%d, v%d, v%d dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE "
                                   "src0_sel:WORD_1 src1_sel:WORD_1" % (spare[i], d[i], x[i]))
                    d, spare = spare, d
                else:
                    for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (d[i], d[i], x[i]))
                    for i in range(4): out.append("v_alignbit_b32 v%d, v%d, v%d, %d" % (d[i], d[i], d[i], 32 - r))
            else:                # c += d; b = rotl(b ^ c, 12 / 7)
                r = 12 if step == 1 else 7
                for i in range(4): out.append("v_add_u32 v%d, v%d, v%d" % (C[i], C[i], d[i]))
                for i in range(4): out.append("v_xor_b32 v%d, v%d, v%d" % (B[i], B[i], C[i]))
                for i in range(4): out.append("v_alignbit_b32 v%d, v%d, v%d, %d" % (B[i], B[i], B[i], 32 - r))
    return out


def main(path):
    g.CLOB = ",".join('"v%d"' % i for i in range(32)) + ',"s20","s21","s22","s23","s24","s25","s26","s27","vcc"'
    variants = {"qr_alignbit": qr(sdwa16=False), "qr_sdwa16": qr(sdwa16=True)}
    for k, v in SINGLE.items():
        variants["1_" + k] = g.single(v)
    src = g.HDR
    calls = []
    for n, ins in variants.items():
        src += g.kernel(n, ins)
        calls.append('    run("%s", k_%s, %d, w);' % (n, n, len(ins)))
    src += g.MAIN % "\n".join(calls)
    open(path, "w").write(src)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "sdwa_bench.hip")
