"""Per-launch listing of the decode calls in a rocprofv3 kernel trace (csv of
the decoder's kernels, as scripts/gpu_r4y.sh writes it): for each call (a
k_stage launch starts one) the kernel, queue, start / end relative to the
call's start and duration in ms.  Usage: dec_launches.py trace.csv [call ...]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_stage" in r["Kernel_Name"]] + [len(rows)]
want = [int(a) for a in sys.argv[2:]] or range(len(starts) - 1)
for c in want:
    i0, i1 = starts[c], starts[c + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in rows[i0:i1])
    print(f"call {c}: {(end - t0) / 1e6:.3f} ms")
    for r in rows[i0:i1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e6
        e = (int(r["End_Timestamp"]) - t0) / 1e6
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("icx::", "")
        print(f"  {name:24s} q{r['Queue_Id']:>3s} {s:8.3f} {e:8.3f} {e - s:7.3f}")
