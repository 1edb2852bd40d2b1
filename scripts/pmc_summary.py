#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into HBM bytes per kernel dispatch.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half
of the bytes of a wide coalesced streaming read -> doubled; WRITE_SIZE (KiB) is
exact for 16-B-per-lane stores (other widths uncalibrated)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, ctr):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, ctr, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != ctr:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name].append(float(r["Counter_Value"]))
    return vals


def main(d, units):
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("icx::"):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / max(1, len(f))
        wb = 1024 * sum(w) / max(1, len(w))
        out[k] = {"dispatches": len(f), "fetch_bytes_per_dispatch_x2": fb, "write_bytes_per_dispatch": wb,
                  "hbm_bytes_per_dispatch": fb + wb}
    short = {k.split("::")[-1].split("<")[0].replace("k_", "").replace("_color", "").replace("_gray", ""): v
             for k, v in out.items()}
    per_unit = {}
    for name, u in units.items():
        if name in short and u > 0:
            per_unit[name] = short[name]["hbm_bytes_per_dispatch"] / u
    res = {"kernels": out, "units_per_dispatch": units, "bytes_per_unit": per_unit}
    json.dump(res, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    # units: work per dispatch in the PMC config (fdct = pixels, huff = scan blocks)
    units = dict(kv.split("=") for kv in sys.argv[2:])
    main(sys.argv[1], {k: float(v) for k, v in units.items()})
