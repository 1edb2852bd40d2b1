#!/usr/bin/env python3
"""Static instruction counts of one kernel of a --save-temps .s file, split
at s_barrier (the phases of a workgroup), by class.  Usage:
  isa_phases.py file.s kernel_substring"""
import re
import sys

src, key = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
seg, segs = {}, []
for l in lines[start:end]:
    t = l.strip()
    if not l.startswith("\t") or t.startswith((".", ";")) or not t:
        continue
    op = t.split()[0]
    cls = "v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_") else \
        "mem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"
    seg[cls] = seg.get(cls, 0) + 1
    seg.setdefault("ops", {})
    seg["ops"][op] = seg["ops"].get(op, 0) + 1
    if op == "s_barrier":
        segs.append(seg)
        seg = {}
segs.append(seg)
for i, s in enumerate(segs):
    top = sorted(s.get("ops", {}).items(), key=lambda kv: -kv[1])[:12]
    print(f"seg {i}: v {s.get('v', 0)} s {s.get('s', 0)} ds {s.get('ds', 0)} mem {s.get('mem', 0)}  ",
          " ".join(f"{k}:{v}" for k, v in top))
