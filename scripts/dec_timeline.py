#!/usr/bin/env python3
"""Timeline of device JPEG decode calls from a rocprofv3 kernel trace
(--kernel-trace --output-format csv): each call starts at a k_stage dispatch;
per call the phases of the critical path - staging + unstuffing + warm-up
walks, the first sync walk, the relaxation (later sync walks), the tail after
the last sync walk - the summed kernel time per family, and how much of the
call's span some decode kernel was running (busy union).  Usage:
dec_timeline.py kernel_trace.csv > summary.json"""
import csv
import json
import sys
from collections import defaultdict


def fam(name):
    return name.split("(")[0].split("<")[0].replace("void ", "").replace("icx::", "").strip()


def union(iv):
    busy, a0, b0 = 0, None, None
    for a, b in sorted(iv):
        if b0 is None or a > b0:
            if b0 is not None:
                busy += b0 - a0
            a0, b0 = a, b
        else:
            b0 = max(b0, b)
    return busy + ((b0 - a0) if b0 is not None else 0)


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_dec" in r["Kernel_Name"] or "k_unstuff" in
            r["Kernel_Name"] or "k_stage" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        f = fam(r["Kernel_Name"])
        if f == "k_stage" and (cur is None or any(fam(x["Kernel_Name"]) != "k_stage" for x in cur)):
            cur = []
            calls.append(cur)
        if cur is not None:
            cur.append(r)
    out = []
    for c in calls:
        ev = [(fam(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "")))
              for r in c]
        t0 = min(e[1] for e in ev)
        t1 = max(e[2] for e in ev)
        syncs = [e for e in ev if e[0] == "k_dec_sync"]
        first_sync = min(syncs, key=lambda e: e[1]) if syncs else None
        last_sync_end = max(e[2] for e in syncs) if syncs else t0
        per = defaultdict(lambda: [0, 0.0])
        for e in ev:
            per[e[0]][0] += 1
            per[e[0]][1] += (e[2] - e[1]) / 1e6
        out.append({
            "span_ms": round((t1 - t0) / 1e6, 3),
            "busy_union_ms": round(union([(e[1], e[2]) for e in ev]) / 1e6, 3),
            "to_first_sync_ms": round(((first_sync[1] if first_sync else t0) - t0) / 1e6, 3),
            "first_sync_ms": round(((first_sync[2] - first_sync[1]) if first_sync else 0) / 1e6, 3),
            "relaxation_ms": round((last_sync_end - (first_sync[2] if first_sync else t0)) / 1e6, 3),
            "sync_launches": len(syncs),
            "tail_after_last_sync_ms": round((t1 - last_sync_end) / 1e6, 3),
            "kernels_ms": {k: {"n": v[0], "ms": round(v[1], 3)} for k, v in sorted(per.items(), key=lambda x: -x[1][1])},
        })
    print(json.dumps({"calls": out}, indent=1))


if __name__ == "__main__":
    main()
