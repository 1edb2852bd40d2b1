#!/usr/bin/env python3
"""FETCH_SIZE x 2 against the known bytes of each calib_fetch kernel.
  calib_summary.py DIR calib.out"""
import csv
import glob
import json
import os
import sys

d, log = sys.argv[1], sys.argv[2]
algo = {}
for line in open(log):
    p = line.split()
    if len(p) >= 3 and p[1] == "algorithmic_bytes":
        algo[p[0]] = int(p[2])
fetch = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") == "FETCH_SIZE":
            fetch.setdefault(r["Kernel_Name"].split("(")[0].replace("void ", ""), []).append(
                float(r["Counter_Value"]) * 1024)
order = ["stream16", "gather_noise", "gather_smooth"]
names = [k for k in fetch if k.startswith(("stream16", "gather_lists"))]
res = {}
gathers = fetch.get("gather_lists", [])
for k, vals in (("stream16", fetch.get("stream16", [])), ("gather_noise", gathers[:1]), ("gather_smooth", gathers[1:2])):
    if vals and k in algo:
        res[k] = {"algorithmic_bytes": algo[k], "fetch_size_bytes": vals[0],
                  "fetch_x2_over_algorithmic": round(2 * vals[0] / algo[k], 4)}
out = {"source": "rocprofv3 --pmc FETCH_SIZE of image-compression_amd/lib/calib_fetch (scripts/calib_fetch.hip)",
       "kernels": res}
json.dump(out, open(os.path.join(d, "calib_fetch_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
