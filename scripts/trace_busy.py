#!/usr/bin/env python3
"""Kernel-trace timeline summary (rocprofv3 --kernel-trace --output-format csv):
per kernel family the summed duration, and the union of busy intervals
against the wall span of the traced dispatches (idle = gaps where no kernel
runs).  Usage: trace_busy.py kernel_trace.csv [name_filter]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    iv = []
    fam = defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r["Kernel_Name"]
        if filt not in name:
            continue
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv.append((a, b))
        k = name.split("(")[0].split("<")[0].replace("void ", "").strip()
        fam[k][0] += 1
        fam[k][1] += (b - a) / 1e6
    iv.sort()
    busy, cur_a, cur_b = 0, None, None
    for a, b in iv:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    span = (iv[-1][1] - iv[0][0]) if iv else 0
    print(json.dumps({"dispatches": len(iv), "span_ms": round(span / 1e6, 3), "busy_union_ms": round(busy / 1e6, 3),
                      "kernels_ms": {k: {"n": v[0], "ms": round(v[1], 3)} for k, v in
                                     sorted(fam.items(), key=lambda x: -x[1][1])}}, indent=1))


if __name__ == "__main__":
    main()
