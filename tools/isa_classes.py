#!/usr/bin/env python3
"""Instruction-class census of one gfx950 kernel from its assembly (hipcc
--cuda-device-only -S): every basic block with the loop depth the compiler
annotates, instructions bucketed into the classes that matter for this
VALU-issue-bound kernel, and the dynamic count per wave
under given trip counts (depth-1 loop x trips1, depth-2 loop x trips2).

    python3 tools/isa_classes.py <file.s> <symbol> [trips_depth1 trips_depth2]
            [--cold LABEL,...]

Classes: ChaCha ARX (v_add_u32 / v_xor_b32 / v_alignbit_b32 / v_bitop3 /
v_perm), Poly1305 multiply (v_mad_u64_u32 / v_mul_*), carries (v_add_co /
v_addc_co / v_sub_co ...), other VALU, DPP / cross-lane (ds_bpermute,
v_readlane, dpp forms), LDS, VMEM (global / buffer incl. LDS-DMA), SALU,
waits / branches.  Blocks listed with --cold (rare paths: partial tiles,
failed tags) are reported but not counted in the dynamic total."""
import collections
import json
import re
import sys


def classify(op, line):
    if op.startswith("ds_bpermute") or op.startswith("v_readlane") or op.startswith("v_readfirstlane") \
            or op.startswith("v_writelane") or "dpp" in line or "row_" in line or "quad_perm" in line:
        return "cross_lane"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt") or op.startswith("s_cbranch") or op.startswith("s_branch") \
            or op.startswith("s_barrier") or op.startswith("s_nop") or op.startswith("s_endpgm"):
        return "wait_branch"
    if op.startswith("s_"):
        return "salu"
    if op in ("v_add_u32_e32", "v_add_u32_e64", "v_xor_b32_e32", "v_xor_b32_e64", "v_alignbit_b32",
              "v_bitop3_b32", "v_perm_b32", "v_xad_u32", "v_add3_u32", "v_xor3_b32", "v_or3_b32",
              "v_add_u32", "v_xor_b32"):
        return "arx"
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mul_") or op.startswith("v_mad_u32"):
        return "mul"
    if "_co_" in op or op.startswith("v_addc") or op.startswith("v_subb") or op.endswith("_co_u32_e32") \
            or op.endswith("_co_u32_e64") or op.startswith("v_cndmask"):
        return "carry_select"
    if op.startswith("v_"):
        return "valu_other"
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cold = set()
    for a in sys.argv[1:]:
        if a.startswith("--cold="):
            cold = set(a.split("=", 1)[1].split(","))
    path, sym = args[0], args[1]
    trips = [1, int(args[2]) if len(args) > 2 else 1, int(args[3]) if len(args) > 3 else 1]
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(sym + ":"))
    blocks = []  # (label, depth, Counter)
    cur, depth = "entry", 0
    counts = collections.Counter()
    ops = collections.Counter()
    for l in text[start + 1:]:
        if l.startswith(".Lfunc_end") or "s_endpgm" in l:
            if "s_endpgm" in l:
                counts["wait_branch"] += 1
            break
        m = re.match(r"^(\.LBB\w+):(.*)", l)
        if m:
            blocks.append((cur, depth, counts, ops))
            cur, counts, ops = m.group(1), collections.Counter(), collections.Counter()
            ds = [int(x) for x in re.findall(r"Depth=(\d+)", m.group(2))]
            depth = max(ds) if ds else 0
            continue
        s = l.strip()
        if s.startswith(";") and "Depth=" in s and not counts:  # "=>This Inner Loop Header: Depth=N"
            depth = max([depth] + [int(x) for x in re.findall(r"Depth=(\d+)", s)])
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        c = classify(op, s)
        if c == "other":
            continue
        counts[c] += 1
        ops[op] += 1
    blocks.append((cur, depth, counts, ops))
    dyn = collections.Counter()
    static = collections.Counter()
    per_depth = collections.defaultdict(collections.Counter)
    hot_ops = collections.Counter()
    by_class = collections.defaultdict(collections.Counter)
    for label, d, c, o in blocks:
        static.update(c)
        per_depth[d].update(c)
        if label in cold:
            continue
        mult = trips[min(d, 2)]
        for k, v in c.items():
            dyn[k] += v * mult
        for k, v in o.items():
            hot_ops[k] += v * mult
            by_class[classify(k, k)][k] += v * mult
    valu = sum(v for k, v in dyn.items() if k in ("arx", "mul", "carry_select", "valu_other", "cross_lane"))
    out = {"symbol": sym, "trips": {"depth1": trips[1], "depth2": trips[2]},
           "static_by_class": dict(static),
           "static_by_depth": {str(d): dict(c) for d, c in sorted(per_depth.items())},
           "dynamic_per_wave": dict(dyn), "dynamic_valu_per_wave": valu,
           "top_ops_dynamic": dict(hot_ops.most_common(40)),
           "ops_by_class_dynamic": {c: dict(o.most_common()) for c, o in sorted(by_class.items())},
           "cold_blocks": sorted(cold)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
