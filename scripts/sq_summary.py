#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 PMC counters (all dispatches), per library build."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    out = {}
    for lib in sorted(os.listdir(d)):
        p = os.path.join(d, lib)
        if not os.path.isdir(p):
            continue
        acc = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if not k.startswith("icx::"):
                    continue
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        out[lib] = acc
        print(f"== {lib}")
        for k, v in sorted(acc.items()):
            print(f"  {k}")
            for c, x in sorted(v.items()):
                print(f"      {c:24s} {x:16.0f}")
    return out


if __name__ == "__main__":
    main(sys.argv[1])
