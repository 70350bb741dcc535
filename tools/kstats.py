"""Per-step kernel breakdown from a rocprofv3 kernel trace (host-side analysis helper).

usage: python tools/kstats.py gpurun_out/prof/run_kernel_trace.csv [--marker adamw_sched] [--top 40] [--shapes]
Takes the span between the last two launches of ``marker`` (one train step) and aggregates by kernel.
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([^(]*?(?:<[^()]*>)?)\(", n)
    return (m.group(1) if m else n)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_sched")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--shapes", action="store_true")
    a = ap.parse_args()
    r = sorted(csv.DictReader(open(a.trace)), key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(r) if a.marker in x["Kernel_Name"]]
    seg = r[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else r
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for x in seg:
        d = int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
        k = short(x["Kernel_Name"])
        if a.shapes:
            k += f" grid={int(x['Grid_Size_X']) // int(x['Workgroup_Size_X'])}x{x['Grid_Size_Y']}x{x['Grid_Size_Z']}"
        agg[k][0] += d
        agg[k][1] += 1
    busy = sum(v[0] for v in agg.values())
    print(f"step wall {(t1 - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, {len(seg)} launches")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{v[0] / 1e3:9.1f} us {100 * v[0] / busy:5.1f}% n={v[1]:4d} avg={v[0] / v[1] / 1e3:7.1f}  {k}")


if __name__ == "__main__":
    main()
