"""Per-kernel (name + grid) time difference of one train step between two rocprofv3 kernel traces.

usage: python tools/kdiff.py NEW_trace.csv OLD_trace.csv [--marker adamw_sched] [--top 30]
"""
import argparse
import collections
import csv
import re


def step(path, marker):
    r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(r) if marker in x["Kernel_Name"]]
    seg = r[idx[-2] + 1: idx[-1] + 1]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for x in seg:
        n = re.sub(r"\(anonymous namespace\)::", "", x["Kernel_Name"])
        n = re.sub(r"^void ", "", n).split("(")[0][:48]
        g = int(x["Grid_Size_X"]) // int(x["Workgroup_Size_X"])
        k = f"{n} g={g}x{x['Grid_Size_Y']}"
        agg[k][0] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
        agg[k][1] += 1
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("new")
    ap.add_argument("old")
    ap.add_argument("--marker", default="adamw_sched")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    n, o = step(a.new, a.marker), step(a.old, a.marker)
    tn, to = sum(v[0] for v in n.values()), sum(v[0] for v in o.values())
    print(f"new {tn:.1f} us ({sum(v[1] for v in n.values())} launches)  old {to:.1f} us "
          f"({sum(v[1] for v in o.values())} launches)  diff {tn - to:+.1f} us")
    keys = set(n) | set(o)
    rows = sorted(keys, key=lambda k: -abs(n.get(k, [0, 0])[0] - o.get(k, [0, 0])[0]))
    for k in rows[: a.top]:
        nv, ov = n.get(k, [0.0, 0]), o.get(k, [0.0, 0])
        print(f"{nv[0] - ov[0]:+9.1f} us  new {nv[0]:8.1f} (n={nv[1]:3d})  old {ov[0]:8.1f} (n={ov[1]:3d})  {k}")


if __name__ == "__main__":
    main()
