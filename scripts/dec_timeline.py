#!/usr/bin/env python3
"""Timeline of device JPEG decode calls from a rocprofv3 kernel trace
(--kernel-trace --output-format csv).  A call starts at its k_stage (device
inputs: header gather) or k_unstuff_count dispatch.  Per call:
  * the phases of the relaxation - to the first sync walk, the first sync
    walk, the later sync walks, the tail after the last one;
  * per queue (HIP stream): the serial chain of dispatches in order, each
    with its start / end relative to the call, its duration and the gap
    before it on that queue, consecutive dispatches of one family merged;
    the queue's busy union;
  * per kernel family: summed dispatch time AND the time it ran alone
    (`alone_ms`: no decode kernel of another family running) against the
    time it shared the chip (`shared_ms`) - a dispatch that overlaps another
    queue's long kernel (e.g. an 18-image k_dec_dc launched beside a
    1000-image k_dec_write) shows a long duration that is mostly waiting for
    CUs, not work (profiles/NOTES.md §10);
  * the critical path as the busy union of all queues against the span
    (idle = host round trips).
Usage: dec_timeline.py kernel_trace.csv > summary.json"""
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


def alone_shared(ev):
    """Per family: time running with no other family active / with others."""
    pts = sorted({t for e in ev for t in (e[1], e[2])})
    alone, shared = defaultdict(float), defaultdict(float)
    for a, b in zip(pts, pts[1:]):
        act = {e[0] for e in ev if e[1] <= a and e[2] >= b}
        for f in act:
            (alone if len(act) == 1 else shared)[f] += (b - a) / 1e6
    return alone, shared


def queue_chain(qev, t0):
    chain, prev_end = [], None
    for f, a, b, _, grid in sorted(qev, key=lambda e: e[1]):
        gap = 0.0 if prev_end is None else max(0.0, (a - prev_end) / 1e6)
        if chain and chain[-1]["kernel"] == f and gap < 0.005:
            chain[-1]["end_ms"] = round((b - t0) / 1e6, 3)
            chain[-1]["ms"] = round(chain[-1]["ms"] + (b - a) / 1e6, 3)
            chain[-1]["n"] += 1
        else:
            chain.append({"kernel": f, "start_ms": round((a - t0) / 1e6, 3), "end_ms": round((b - t0) / 1e6, 3),
                          "ms": round((b - a) / 1e6, 3), "gap_before_ms": round(gap, 3), "n": 1, "grid": grid})
        prev_end = b
    return chain


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_dec" in r["Kernel_Name"] or "k_unstuff" in
            r["Kernel_Name"] or "k_stage" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls, cur, last = [], None, None
    for r in rows:
        f = fam(r["Kernel_Name"])
        if (f == "k_stage" and last != "k_stage") or (f == "k_unstuff_count" and last != "k_stage"):
            cur = []
            calls.append(cur)
        if cur is not None:
            cur.append(r)
        last = f
    out = []
    for c in calls:
        ev = [(fam(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
               r.get("Queue_Id", r.get("Stream_Id", "")), f'{r.get("Grid_Size_X", "")}x{r.get("Grid_Size_Y", "")}')
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
        alone, shared = alone_shared(ev)
        queues = defaultdict(list)
        for e in ev:
            queues[e[3]].append(e)
        busy = union([(e[1], e[2]) for e in ev])
        out.append({
            "span_ms": round((t1 - t0) / 1e6, 3),
            "busy_union_ms": round(busy / 1e6, 3),
            "idle_ms": round((t1 - t0 - busy) / 1e6, 3),
            "to_first_sync_ms": round(((first_sync[1] if first_sync else t0) - t0) / 1e6, 3),
            "first_sync_ms": round(((first_sync[2] - first_sync[1]) if first_sync else 0) / 1e6, 3),
            "relaxation_ms": round((last_sync_end - (first_sync[2] if first_sync else t0)) / 1e6, 3),
            "sync_launches": len(syncs),
            "tail_after_last_sync_ms": round((t1 - last_sync_end) / 1e6, 3),
            "kernels_ms": {k: {"n": v[0], "ms": round(v[1], 3), "alone_ms": round(alone[k], 3),
                               "shared_ms": round(shared[k], 3)}
                           for k, v in sorted(per.items(), key=lambda x: -x[1][1])},
            "queues": {str(q): {"busy_ms": round(union([(e[1], e[2]) for e in qe]) / 1e6, 3),
                                "chain": queue_chain(qe, t0)} for q, qe in sorted(queues.items())},
        })
    print(json.dumps({"calls": out}, indent=1))


if __name__ == "__main__":
    main()
