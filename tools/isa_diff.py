#!/usr/bin/env python3
"""Per-kernel ISA comparison of two device-assembly files (hipcc
--cuda-device-only -S -g0): each function's instruction text, with comments
and function-numbered labels normalised, is hashed; kernels present in both
files are reported as same / CHANGED, then those only in one.  Used to show
that a source clean-up left the shipping kernels' machine code unchanged.

usage: isa_diff.py OLD.s NEW.s [--show NAME_SUBSTRING]
"""
import hashlib
import re
import sys


def functions(path):
    out, name, body = {}, None, []
    for line in open(path):
        s = line.rstrip("\n")
        m = re.match(r"\s*\.type\s+([^,]+),@function", s)
        if m:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if s.startswith(".Lfunc_end"):
            out[name] = body
            name = None
            continue
        s = s.split(";")[0].rstrip()
        if not s.strip() or s.strip().startswith("."):
            if not re.match(r"^\.L\w+:", s):
                continue
        s = re.sub(r"\.LBB\d+_(\d+)", r".LBB_\1", s)
        s = re.sub(r"\.Ltmp\d+", ".Ltmp", s)
        body.append(s)
    return out


def main():
    a, b = functions(sys.argv[1]), functions(sys.argv[2])
    show = sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--show" else None
    same = changed = 0
    for k in sorted(set(a) & set(b)):
        ha = hashlib.sha1("\n".join(a[k]).encode()).hexdigest()[:12]
        hb = hashlib.sha1("\n".join(b[k]).encode()).hexdigest()[:12]
        if ha == hb:
            same += 1
        else:
            changed += 1
            print(f"CHANGED {k} ({len(a[k])} -> {len(b[k])} lines)")
            if show and show in k:
                import difflib
                sys.stdout.writelines(l + "\n" for l in difflib.unified_diff(a[k], b[k], lineterm="", n=2))
    for k in sorted(set(a) - set(b)):
        print(f"only in old: {k}")
    for k in sorted(set(b) - set(a)):
        print(f"only in new: {k}")
    print(f"{same} same, {changed} changed, {len(set(a) - set(b))} removed, {len(set(b) - set(a))} added")


if __name__ == "__main__":
    main()
