#!/usr/bin/env python3
"""Instruction mix of kernels in a hipcc --save-temps .s: python tools/isa_stats.py file.s [name-regex]."""
import re
import sys

PATS = {"valu": r"^\s+v_", "pk": r"^\s+v_pk_", "salu": r"^\s+s_(?!waitcnt|barrier|cbranch|branch|endpgm|nop)",
        "vmem": r"^\s+(buffer|global|flat)_", "lds": r"^\s+ds_", "saveexec": r"s_and_saveexec"}
s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r".")
for m in re.finditer(r"^(_Z\w+):\s*;[^\n]*\n(.*?)^\.Lfunc_end\d+:", s, re.M | re.S):
    name, body = m.group(1), m.group(2)
    if not pat.search(name):
        continue
    meta = re.search(r"\.name:\s+" + re.escape(name) + r"\b", s)
    blk = s[s.rfind("- .agpr_count", 0, meta.start()) if meta else 0: meta.start() if meta else 0]
    meta_v = {k: (re.findall(r"\." + k + r":\s+(\d+)", blk) or ["?"])[-1] for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count")}
    cnt = {k: len(re.findall(p, body, re.M)) for k, p in PATS.items()}
    print(f"{name[:64]:64s} " + " ".join(f"{k} {v}" for k, v in meta_v.items()) + " " + " ".join(f"{k} {v}" for k, v in cnt.items()))
