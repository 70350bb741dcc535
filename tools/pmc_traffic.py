"""Per-kernel HBM traffic from separate rocprofv3 ``--pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` passes (host-side helper).

usage: python tools/pmc_traffic.py gpurun_out/pmc --fetch p3 --write p4 --match "conv3x3_halo9b<false, 2, 0>" \
           --algorithmic 276824064 --label "..." --round 5 --out profiles/r5_halo9b_fwd_traffic.json

FETCH_SIZE is doubled (gfx950: it reports half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md HBM
section); WRITE_SIZE is taken as is (exact for 16-B stores).  Both counters are in KB per dispatch.  Averages over
every dispatch of the matching kernel (exact name match after stripping ``void`` / the anonymous namespace / the
argument list), separately per ``Grid_Size`` when ``--grid`` is given.
"""
import argparse
import csv
import glob
import json
import os
import re


def _name(k):
    return re.sub(r"\(anonymous namespace\)::", "", k).replace("void ", "").split("(")[0].strip()


def per_dispatch(d, counter, match, grid):
    tot = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")) + glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if _name(r["Kernel_Name"]) != match or r["Counter_Name"] != counter:
                continue
            if grid and int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) != grid:
                continue
            tot[r["Dispatch_Id"]] = tot.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(tot.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--fetch", default="p3")
    ap.add_argument("--write", default="p4")
    ap.add_argument("--match", required=True, action="append", help="kernel name; repeat to sum kernels per launch")
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--algorithmic", type=float, required=True, help="algorithmic bytes per launch")
    ap.add_argument("--label", default="")
    ap.add_argument("--round", type=int, default=5)
    ap.add_argument("--out")
    a = ap.parse_args()
    fkb = wkb = 0.0
    counts = []
    for m in a.match:
        fv = per_dispatch(os.path.join(a.dir, a.fetch), "FETCH_SIZE", m, a.grid)
        wv = per_dispatch(os.path.join(a.dir, a.write), "WRITE_SIZE", m, a.grid)
        if not fv or not wv:
            raise SystemExit(f"no dispatches of {m!r} (fetch {len(fv)}, write {len(wv)})")
        fkb += sum(fv) / len(fv)
        wkb += sum(wv) / len(wv)
        counts.append([len(fv), len(wv)])
    rd, wr = 2 * fkb * 1024, wkb * 1024
    res = {
        "kernel_id": a.match if len(a.match) > 1 else a.match[0],
        "kernel": a.label or " + ".join(a.match),
        "passes": f"rocprofv3 --pmc FETCH_SIZE ({a.fetch}) and --pmc WRITE_SIZE ({a.write}), separate runs, round {a.round}",
        "fetch_size_kb_per_launch": fkb,
        "write_size_kb_per_launch": wkb,
        "correction": "gfx950: FETCH_SIZE reports half the bytes of 16-B/lane streaming reads -> x2; WRITE_SIZE exact "
                      "for 16-B stores (MI355X_MICROARCH.md HBM section)",
        "hbm_read_bytes": rd,
        "hbm_write_bytes": wr,
        "traffic_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": a.algorithmic,
        "traffic_over_algorithmic": (rd + wr) / a.algorithmic,
        "dispatches": counts,
    }
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
