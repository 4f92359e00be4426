#!/usr/bin/env python3
"""Histogram of instruction classes per basic block of one kernel in a hipcc --save-temps .s file.

Usage: tools/isa_loops.py file.s <kernel-substring> [min_block_len]
Prints each block (label, #instrs, class counts) and marks blocks that end in a backward branch (loops).
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_"):
        if "_f64" in op or op.startswith("v_fma_f64") or op.endswith("f64_e64"):
            return "valu64"
        if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            return "lane"
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, kname = sys.argv[1], sys.argv[2]
    minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and kname in l.split(":")[0]:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    order = [cur]
    for l in lines[start + 1:]:
        if re.match(r"^_Z\S*:", l) or l.startswith("\t.section") or ".Lfunc_end" in l:
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        blocks[cur].append(s.split()[0] if s.split() else s)
    pos = {b: i for i, b in enumerate(order)}
    tot = Counter()
    for b in order:
        ins = blocks[b]
        c = Counter(classify(o) for o in ins)
        tot.update(c)
        back = ""
        last = " ".join(ins[-2:])
        for o in ins[-2:]:
            pass
        # detect a backward branch target
        raw = [l for l in ins if l.startswith(("s_cbranch", "s_branch"))]
        if len(ins) >= minlen:
            print(f"{b:28s} n={len(ins):5d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
    print("TOTAL", " ".join(f"{k}={v}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
