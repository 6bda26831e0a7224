#!/usr/bin/env python3
"""Per-opcode census of one kernel in a hipcc -S (gfx950) assembly file.

usage: asm_census.py FILE.s SYMBOL_SUBSTRING [--blocks]
Prints the function's instruction counts by opcode and by class (v_mad_u64_u32, other VALU,
SALU, memory, LDS, branch, s_nop), and with --blocks the same per basic block (label), so the
hot loop's blocks can be read off (they are the ones the back edge of the main loop spans).
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op == "v_mad_u64_u32":
        return "mad_u64_u32"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    blocks_mode = "--blocks" in sys.argv
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S*):", l)
        if m and sym in m.group(1):
            start = i
            break
    if start is None:
        sys.exit("symbol not found")
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = Counter()
    for l in lines[start + 1:]:
        if l.startswith("\t.size") or l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = Counter()
            continue
        s = l.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        if not re.match(r"^[sv]_|^(global|buffer|flat|ds|scratch)_", op):
            continue
        blocks[cur][op] += 1
    total = Counter()
    for c in blocks.values():
        total.update(c)
    def report(name, c):
        cls = Counter()
        for op, k in c.items():
            cls[classify(op)] += k
        print("== %s: %d instructions" % (name, sum(c.values())))
        print("   classes: " + ", ".join("%s %d" % kv for kv in cls.most_common()))
        print("   opcodes: " + ", ".join("%s %d" % kv for kv in c.most_common()))
    report("function total", total)
    if blocks_mode:
        for name, c in blocks.items():
            if sum(c.values()):
                report(name, c)


if __name__ == "__main__":
    main()
