#!/usr/bin/env python3
"""Instruction-issue summary for bench.py's roofline object: per-kernel VALU /
SALU / LDS instructions and waves per unit of work, from a rocprofv3 SQ
counter run of the headline workload (scripts/gpu_sq.sh with SQ_ARGS from
this file's docstring).  Units: fdct = pixels, huff = scan blocks coded.

Usage: sq_issue.py <sq run dir> <frames> <huff blocks coded> > profiles/sq_issue_summary.json
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from sq_summary import main as summarize  # noqa: E402


def run(d, frames, huff_blocks):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        acc = summarize(d)["libicx"]
    units = {"icx::k_fdct_color<true>": frames * 3840 * 2160, "icx::k_huff": huff_blocks}
    import os
    out = {"source": "rocprofv3 SQ counters, bench.py headline workload",
           "tree_commit": os.environ.get("ICX_COMMIT", "unknown"), "units": {}, "per_unit": {}}
    for k, u in units.items():
        v = acc[k]
        name = "fdct" if "fdct" in k else "huff"
        out["units"][name] = u
        out["per_unit"][name] = {c: v.get(c, 0.0) / u for c in
                                 ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES")}
    return out


if __name__ == "__main__":
    print(json.dumps(run(sys.argv[1], int(sys.argv[2]), float(sys.argv[3])), indent=1))
