"""Summarise rocprofv3 --pmc counter CSVs per kernel (host-side helper).

usage: python tools/pmc_sum.py gpurun_out/pmc [--match conv3x3_halo]
Prints, per kernel name and counter, the mean per dispatch over all dispatches in all passes.
"""
import argparse
import collections
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--match", default="")
a = ap.parse_args()
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.dir, "p*", "*counter_collection.csv"))):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).replace("void ", "").split("(")[0]
        if a.match and a.match not in n:
            continue
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = n
    for (disp, cname), v in per.items():
        vals[names[disp]][cname].append(v)
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
