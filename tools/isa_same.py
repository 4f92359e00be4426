#!/usr/bin/env python3
"""isa_same.py BEFORE.s AFTER.s -- which kernels of AFTER have an instruction stream identical to a
kernel of BEFORE (device assembly from `hipcc --cuda-device-only -S`).  Block labels are renumbered
and the kernel's own (mangled) name is masked, so a kernel whose template parameters were dropped
still matches.  Used for the round-5 removal of measured-and-rejected variants."""
import re
import subprocess
import sys


def funcs(path):
    out, cur, buf = {}, None, []
    for line in open(path).read().split("\n"):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, buf = m.group(1), []
            continue
        if cur and re.match(r"^\s*\.Lfunc_end", line):
            out[cur] = buf
            cur = None
            continue
        if cur:
            t = line.split(";")[0].rstrip()
            if t.strip():
                buf.append(t)
    return out


def norm(name, lines):
    labels, out = {}, []
    for line in lines:
        for lab in re.findall(r"\.LBB\d+_\d+", line):
            labels.setdefault(lab, f"L{len(labels)}")
        line = re.sub(r"\.LBB\d+_\d+", lambda x: labels[x.group(0)], line)
        out.append(line.replace(name, "KERNEL"))
    return out


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


def main():
    before, after = funcs(sys.argv[1]), funcs(sys.argv[2])
    nb = {k: norm(k, v) for k, v in before.items()}
    same = 0
    for k, v in after.items():
        body = norm(k, v)
        hit = next((b for b, bb in nb.items() if bb == body), None)
        same += hit is not None
        print(("SAME  " if hit else "DIFF  ") + demangle(k) + (f"   == {demangle(hit)}" if hit else ""))
    print(f"{same} of {len(after)} kernels identical; {len(before)} kernels before")


if __name__ == "__main__":
    main()
