#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of one bench.py run into HBM bytes per unit
of work, next to the algorithmic bytes the library counted in the same run.

  pmc_summary.py DIR BENCH_JSON

DIR holds one rocprofv3 output per counter (DIR/FETCH_SIZE, DIR/WRITE_SIZE);
BENCH_JSON is the JSON line of the same command (run with --warmup 0 --steps 1
so that every icx:: dispatch of the process is a timed one; the line's
"kernels" give units and algorithmic bytes).  gfx950 corrections
(MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) counts half the bytes of a wide
coalesced read -> doubled; profiles/r2/calib_fetch_summary.json shows the
same factor for k_huff's 16-B list gathers.  WRITE_SIZE is exact for 16-B
stores (k_huff's and k_fdct's)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SHORT = {"k_fdct_color": "fdct", "k_fdct_gray": "fdct", "k_huff": "huff", "k_scan": "scan",
         "k_ffscan": "ffscan", "k_stuff": "stuff", "k_resize": "resize"}


def load(d, ctr):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, ctr, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != ctr:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name].append(float(r["Counter_Value"]))
    return vals


def aggregate(out, kern):
    """Bytes per unit of each bench kernel name over every icx:: kernel that
    maps to it (k_fdct_color and k_fdct_gray are both "fdct"; icx_create's
    self-check dispatches each on a 16x16 image, so a name's dispatches are
    not all one kernel's).  The per-kernel entries keep their own bytes;
    their unit ratios are dropped where a name has several kernels."""
    groups = defaultdict(list)
    for k in out:
        short = SHORT.get(k.split("::")[-1].split("<")[0])
        if short:
            groups[short].append(k)
    per_unit, info = {}, {}
    for short, ks in groups.items():
        if short not in kern or not kern[short].get("units"):
            continue
        hb = sum(out[k]["hbm_bytes"] for k in ks)
        ku = kern[short]
        per_unit[short] = hb / ku["units"]
        info[short] = {"kernels": ks, "hbm_bytes": hb, "units": ku["units"], "hbm_bytes_per_unit": per_unit[short]}
        if ku.get("algo_bytes"):
            info[short]["algo_bytes_per_unit"] = ku["algo_bytes"] / ku["units"]
            info[short]["traffic_over_algo"] = hb / ku["algo_bytes"]
        if len(ks) > 1:
            for k in ks:
                for f in ("units", "bench_launches", "hbm_bytes_per_unit", "algo_bytes", "algo_bytes_per_unit",
                          "traffic_over_algo"):
                    out[k].pop(f, None)
                out[k]["bench_kernel"] = short
    return per_unit, info


def main(d, bench_json):
    line = json.loads([l for l in open(bench_json) if l.startswith("{")][-1])
    kern = line["kernels"]
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("icx::"):
            continue
        short = SHORT.get(k.split("::")[-1].split("<")[0])
        f, w = fetch.get(k, []), write.get(k, [])
        fb, wb = 2 * 1024 * sum(f), 1024 * sum(w)
        e = {"dispatches": len(f), "fetch_bytes_x2": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
             "fetch_x2_per_dispatch": [round(2 * 1024 * v) for v in f]}
        if short in kern and kern[short].get("units"):
            ku = kern[short]
            e["units"] = ku["units"]
            e["bench_launches"] = ku["launches"]
            e["hbm_bytes_per_unit"] = (fb + wb) / ku["units"]
            if "algo_bytes" in ku:
                e["algo_bytes"] = ku["algo_bytes"]
                e["algo_bytes_per_unit"] = ku["algo_bytes"] / ku["units"]
                e["traffic_over_algo"] = (fb + wb) / ku["algo_bytes"]
        out[k] = e
    per_unit, info = aggregate(out, kern)
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of: bench.py " +
                     " ".join(sys.argv[3:]), "tree_commit": os.environ.get("ICX_COMMIT", "unknown"),
           "kernels": out, "bench_kernels": info, "bytes_per_unit": per_unit}
    # the file bench.py reads (profiles/pmc_summary.json is a copy of it, not
    # of stdout): "bytes_per_unit" maps the bench's kernel names to HBM bytes
    json.dump(res, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
