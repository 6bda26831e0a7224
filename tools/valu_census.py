#!/usr/bin/env python3
"""Category census of k_accumulate's hot loop from its gfx950 assembly.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I kzg-batch-verification-scheme_amd/csrc \
        -DKZ_CURVE=0 -S --cuda-device-only kzg-batch-verification-scheme_amd/csrc/launch_msm.hip -o /tmp/lm0.s
    python tools/valu_census.py /tmp/lm0.s bls12_381 [mix_rate.txt]

The loop body of one mixed addition is straight-line code in a few basic blocks: the point load
and conditional negation, then the two blocks holding the products (the blocks with >= 300
v_mad_u64_u32 of the static-grid copy of the loop).  Opcodes are grouped by what they do in
field29.hpp / msm.hpp acc_loop29:
  mad           v_mad_u64_u32: the limb products a_i b_j and m_i p_j
  column        per Montgomery column: v_mul_lo_u32 (m = acc p' mod 2^32), v_lshrrev_b64 (acc >>= 29),
                and 2 v_and_b32 per column (m mod 2^29, the output limb)
  carry         the remaining v_and_b32 + v_lshrrev_b32 / v_add3_u32 / v_sub_u32 / v_add_u32 /
                v_lshl_add_u32 / v_alignbit_b32: sub29 / sub3_29 carry passes and the negation
  zero_test     v_cmp*, v_cndmask*, v_bitop3*, v_lshlrev_b16, v_or_b32: is_zero29_mf of P and R
  lane_lds      v_readlane / v_writelane / v_mov / LDS and memory instructions, waitcnt, SALU, branch
  s_nop         hipcc's pad after every VGPR-writing inline-asm statement (4 mads per statement)
With a mix_rate.txt (tools/probes/mix_rate.hip output) each category is also priced by the
measured marginal cost of its opcodes beside mads, giving the share of the loop's issue time.
"""
import re
import sys
from collections import Counter


def blocks(path, sym):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.split(";")[0].rstrip().endswith(":"))
    out, cur, name = [], [], "entry"
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        cur.append(t.split()[0])
    out.append((name, cur))
    return out


def category(op):
    if op == "v_mad_u64_u32":
        return "mad"
    if op.startswith("s_nop"):
        return "s_nop"
    if op in ("v_mul_lo_u32", "v_lshrrev_b64"):
        return "column"
    if op.startswith(("v_cmp", "v_cndmask", "v_bitop3", "v_lshlrev_b16", "v_or_b32")):
        return "zero_test"
    if op.startswith(("v_and_b32", "v_lshrrev_b32", "v_add3_u32", "v_sub_u32", "v_add_u32", "v_lshl_add_u32",
                      "v_alignbit_b32", "v_lshlrev_b32")):
        return "carry"
    return "lane_lds"


def main():
    path, curve = sys.argv[1], sys.argv[2]
    mix = sys.argv[3] if len(sys.argv) > 3 else None
    sym = {"bls12_381": "_ZN5kzgmi12k_accumulateINS_9Bls12_381", "bn254": "_ZN5kzgmi12k_accumulateINS_5Bn254"}[curve]
    n_limbs = 14 if curve == "bls12_381" else 9
    bl = blocks(path, sym)
    # the first copy of the loop: the blocks with >= 300 mads, and the negation block before them
    hot = [i for i, (_, ops) in enumerate(bl) if sum(o == "v_mad_u64_u32" for o in ops) >= 300][:2]
    neg = hot[0] - 1
    while sum(o.startswith("global_load") for o in bl[neg][1]) == 0:
        neg -= 1
    idx = [neg] + hot
    ops = Counter(o for i in idx for o in bl[i][1])
    # 2 v_and per Montgomery column belong to the column steps (m mod 2^29, the output limb)
    nprod = ops["v_mul_lo_u32"] / n_limbs  # one v_mul_lo per low column (+ the zero tests' filters)
    cats = Counter()
    for op, k in ops.items():
        cats[category(op)] += k
    col_and = round(2 * (n_limbs - 0.5) * int(nprod))
    cats["column"] += col_and
    cats["carry"] -= col_and
    valu = sum(k for op, k in ops.items() if op.startswith("v_"))
    print("k_accumulate<%s> hot loop, blocks %s (static-grid copy): %d instructions, %d VALU"
          % (curve, ", ".join(bl[i][0] for i in idx), sum(ops.values()), valu))
    print("  Montgomery reductions in the loop: %.1f (v_mul_lo_u32 / %d limbs)" % (nprod, n_limbs))
    for c in ("mad", "column", "carry", "zero_test", "lane_lds", "s_nop"):
        print("  %-10s %5d" % (c, cats[c]))
    print("  opcodes:", ", ".join("%s %d" % kv for kv in ops.most_common()))
    if mix:
        cost = {}
        for l in open(mix):
            m = re.match(r"^\+8 (\S+)\s+\S+ ns/iter\s+marginal\s+(-?[\d.]+)", l)
            if m:
                cost[m.group(1)] = max(0.0, float(m.group(2)))
            m = re.match(r"^8 mads alone\s+([\d.]+)", l)
            if m:
                cost["v_mad_u64_u32"] = float(m.group(1)) / 8
        # mads at their marginal cost beside mads (the loop's dominant stream), other VALU opcodes
        # the probe does not cover at the median VALU marginal, s_nop at its own (~0.15 ns)
        if "v_mad_u64_u32" in cost:
            cost["v_mad_u64_u32"] = [float(m.group(1)) for m in
                                     (re.match(r"^\+8 v_mad_u64_u32\s+\S+ ns/iter\s+marginal\s+([\d.]+)", l)
                                      for l in open(mix)) if m][0]
        for l in open(mix):
            m = re.match(r"^\+8 s_nop 0\s+\S+ ns/iter\s+marginal\s+(-?[\d.]+)", l)
            if m:
                cost["s_nop"] = max(0.0, float(m.group(1)))
        vmed = sorted(v for k, v in cost.items() if k.startswith("v_"))[len([k for k in cost if k.startswith("v_")]) // 2]

        def price(op):
            for k in sorted(cost, key=len, reverse=True):
                if op.startswith(k):
                    return cost[k]
            return vmed if op.startswith("v_") else None
        tot, unpriced = Counter(), Counter()
        for op, k in ops.items():
            p = price(op)
            c = category(op)
            if p is None:
                unpriced[c] += k
            else:
                tot[c] += p * k
        # the column's v_and are priced like the carry passes' (same opcode)
        pa = price("v_and_b32") or 0.0
        tot["column"] += pa * col_and
        tot["carry"] -= pa * col_and
        s = sum(tot.values())
        print("priced by tools/probes/mix_rate.hip (ns per wave-slot beside mads, 4 waves/SIMD):")
        for c in ("mad", "column", "carry", "zero_test", "lane_lds", "s_nop"):
            print("  %-10s %8.1f ns  %5.1f %%%s" % (c, tot[c], 100 * tot[c] / s if s else 0,
                                                  ("  (+%d unpriced instructions)" % unpriced[c]) if unpriced[c] else ""))


if __name__ == "__main__":
    main()
