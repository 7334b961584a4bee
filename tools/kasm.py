#!/usr/bin/env python3
"""Extract one kernel's ISA from a --save-temps .s file and summarise its
loops: per basic block instruction mix (VALU / LDS / VMEM / waitcnt).
usage: kasm.py FILE.s MANGLED_SUBSTRING [--dump]"""
import re, sys
from collections import Counter
path, key = sys.argv[1], sys.argv[2]
lines, on = [], False
for ln in open(path):
    if not on and re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", ln):
        on = True
    elif on and re.match(r"^\s*\.size\s", ln):
        break
    if on:
        lines.append(ln.rstrip("\n"))
if "--dump" in sys.argv:
    print("\n".join(lines)); sys.exit()
blocks, cur = [], ("entry", [])
for ln in lines:
    m = re.match(r"^(\.LBB\S+):", ln)
    if m:
        blocks.append(cur); cur = (m.group(1), []); continue
    t = ln.strip()
    if t and not t.startswith((";", ".", "//")):
        cur[1].append(t.split()[0])
blocks.append(cur)
for name, ins in blocks:
    c = Counter()
    for op in ins:
        k = ("lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else
             "wait" if op.startswith("s_waitcnt") else "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "other")
        c[k] += 1
    br = [op for op in ins if op.startswith("s_cbranch") or op == "s_branch"]
    print(f"{name:24s} n={len(ins):5d} " + " ".join(f"{k}={c[k]}" for k in ("valu", "lds", "vmem", "wait", "salu")))
