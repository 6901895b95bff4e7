#!/usr/bin/env python3
"""Opcode histogram of a kernel's hottest loop body from an llvm-objdump listing.

    python3 tools/isa/isa_hist.py <listing.s> <kernel-substring> [--all]

The loop is the instruction range [target, branch] of the backward s_cbranch / s_branch that spans
the most instructions (the ladder's step loop); --all histograms the whole kernel instead."""
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
    if "--all" not in sys.argv:
        best = None
        for k, (addr, op, ln) in enumerate(insns):
            b = BR.match(ln)
            if not b:
                continue
            # llvm-objdump prints the branch offset in dwords relative to the next instruction
            tgt = addr + 4 + 4 * int(b.group(2)) if int(b.group(2)) < 32768 else addr + 4 + 4 * (int(b.group(2)) - 65536)
            if tgt < addr:
                lo = next(i for i, x in enumerate(insns) if x[0] >= tgt)
                if best is None or k - lo > best[1] - best[0]:
                    best = (lo, k)
        if best:
            body = insns[best[0]:best[1] + 1]
    h = Counter(op for _, op, _ in body)
    total = sum(h.values())
    print(f"{name}: {total} instructions in the {'kernel' if body is insns else 'loop body'}")
    for op, c in h.most_common():
        print(f"{c:6d}  {100.0 * c / total:5.1f}%  {op}")


if __name__ == "__main__":
    main()
