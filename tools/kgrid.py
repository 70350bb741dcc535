"""Per-(kernel, grid) aggregation of one train step from a rocprofv3 kernel trace (host-side helper).

usage: python tools/kgrid.py gpurun_out/prof/run_kernel_trace.csv [--match substr[,substr]] [--marker adamw]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--match", default="")
ap.add_argument("--marker", default="adamw")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
lo, hi = (idx[-2], idx[-1]) if len(idx) >= 2 else (0, len(rows) - 1)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[lo + 1:hi + 1]:
    n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).replace("void ", "")
    if a.match and not any(m in n for m in a.match.split(",")):
        continue
    n = n.split("(")[0][:48]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    key = (n, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[key][0] += 1
    agg[key][1] += d
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{v[1]:8.1f} us n={v[0]:3d} avg={v[1] / v[0]:7.1f}  {k[0]:48s} {k[1]}x{k[2]}x{k[3]}")
