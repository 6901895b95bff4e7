#!/usr/bin/env python3
"""Opcode histogram of a kernel's hottest loop body from an llvm-objdump listing.

    python3 tools/isa/isa_hist.py <listing.s> <kernel-substring> [--all | --loops]

The loop is the instruction range [target, branch] of the backward s_cbranch / s_branch that spans
the most instructions (the ladder's step loop); --all histograms the whole kernel instead; --loops
lists every loop (start address, instructions, scalar / vector / 64-bit mad / DPP / readlane counts)."""
import re
import sys
from collections import Counter

INSN = re.compile(r"^\s+([0-9a-z_]+)(?:\s|$)")
ADDR = re.compile(r"//\s*([0-9A-F]+):")
BR = re.compile(r"^\s+(s_cbranch_\w+|s_branch)\s+(\d+)")


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if re.match(r"^[0-9a-f]+ <.*>:", line):
            on = name in line
            continue
        if on:
            out.append(line.rstrip("\n"))
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, name)
    insns = []  # (addr, opcode, line)
    for ln in lines:
        m, a = INSN.match(ln), ADDR.search(ln)
        if m and a and not m.group(1).startswith("."):
            insns.append((int(a.group(1), 16), m.group(1), ln))
    body = insns
    loops = []
    for k, (addr, op, ln) in enumerate(insns):
        b = BR.match(ln)
        if not b:
            continue
        # llvm-objdump prints the branch offset in dwords relative to the next instruction
        tgt = addr + 4 + 4 * int(b.group(2)) if int(b.group(2)) < 32768 else addr + 4 + 4 * (int(b.group(2)) - 65536)
        if tgt < addr:
            loops.append((next(i for i, x in enumerate(insns) if x[0] >= tgt), k))
    if "--loops" in sys.argv:
        for lo, hi in sorted(loops):
            c = Counter(op for _, op, _ in insns[lo:hi + 1])
            n = lambda pre: sum(v for o, v in c.items() if o.startswith(pre))
            print(f"{insns[lo][0]:#x}: {hi - lo + 1:5d} insns  salu {n('s_'):5d}  valu {n('v_'):5d}  "
                  f"mad64 {c['v_mad_u64_u32'] + c['v_mad_i64_i32']:4d}  dpp {c['v_mov_b32_dpp']:3d}  "
                  f"readlane {c['v_readlane_b32']:3d}")
        return
    if "--all" not in sys.argv and loops:
        lo, hi = max(loops, key=lambda x: x[1] - x[0])
        body = insns[lo:hi + 1]
    h = Counter(op for _, op, _ in body)
    total = sum(h.values())
    print(f"{name}: {total} instructions in the {'kernel' if body is insns else 'loop body'}")
    for op, c in h.most_common():
        print(f"{c:6d}  {100.0 * c / total:5.1f}%  {op}")


if __name__ == "__main__":
    main()
