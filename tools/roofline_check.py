"""Cross-check bench.py's live roofline timings against the rocprofv3 kernel trace of the same command.

usage: python tools/roofline_check.py gpurun_out/prof/run_kernel_trace.csv [--n 20] [--bench gpurun_out/prof/bench.json]

bench.py's conv_roofline() issues 3 warm-up + 20 timed launches of each roofline problem (8x256^2, 128 -> 128) after
the train and sampler legs, so they are the LAST launches of their kernel at that grid in the trace:
  fwd    conv3x3_halo9b<false, 2, 0>, 2048 workgroups x 256 threads
  dgrad  conv3x3_halo9b<false, 0, 0>, 2048 x 256
  wgrad  wgrad_halo_kernel<2> (its grid) + the wgrad_reduce2 launch that follows each one
Prints per problem the trace's mean / min / max duration (us) of those launches and, with --bench, the HIP-event
time bench.py measured for the same launches (bench.py times each launch after a 512 MB cache-evicting write).
"""
import argparse
import csv
import json
import re

GF = 2.0 * 8 * 256 * 256 * 128 * 128 * 9 / 1e9


def _name(k):
    return re.sub(r"\(anonymous namespace\)::", "", k).replace("void ", "").split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--bench", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        r["name"] = _name(r["Kernel_Name"])
        r["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    bench = {}
    if a.bench:
        with open(a.bench) as f:
            line = [ln for ln in f if ln.startswith("{")][-1]
        j = json.loads(line)
        bench = {"fwd": j["roofline"]["kernel_ms"] * 1e3, "dgrad": j["roofline_backward"]["dgrad"]["kernel_ms"] * 1e3,
                 "wgrad": j["roofline_backward"]["wgrad"]["kernel_ms"] * 1e3}
    for prob, kname in (("fwd", "conv3x3_halo9b<false, 2, 0, 16>"), ("dgrad", "conv3x3_halo9b<false, 0, 0, 16>")):
        sel = [r for r in rows if r["name"] == kname and int(r["Grid_Size_X"]) == 2048 * 256 and r["Grid_Size_Y"] == "1"]
        d = [r["us"] for r in sel[-a.n:]]
        ev = f", bench.py HIP events {bench[prob]:.1f} us" if prob in bench else ""
        print(f"{prob:6s} {kname} (8x256x256x128->128) last {len(d)} launches: mean {sum(d) / len(d):.1f} us "
              f"({GF / (sum(d) / len(d)) * 1e3:.0f} TF/s), min {min(d):.1f}, max {max(d):.1f}{ev}")
    idx = [i for i, r in enumerate(rows) if r["name"] == "wgrad_halo_kernel<2, false>"]
    grid = rows[idx[-1]]["Grid_Size_X"]
    idx = [i for i in idx if rows[i]["Grid_Size_X"] == grid][-a.n:]
    kern, red = [], []
    for i in idx:
        kern.append(rows[i]["us"])
        nxt = next((rows[j] for j in range(i + 1, min(i + 4, len(rows))) if rows[j]["name"] == "wgrad_reduce2"), None)
        red.append(nxt["us"] if nxt else 0.0)
    tot = [k + r for k, r in zip(kern, red)]
    ev = f", bench.py HIP events {bench['wgrad']:.1f} us" if "wgrad" in bench else ""
    print(f"wgrad  wgrad_halo_kernel<2, false> + wgrad_reduce2 last {len(tot)}: kernel mean {sum(kern) / len(kern):.1f} us, "
          f"reduce mean {sum(red) / len(red):.1f} us, sum {sum(tot) / len(tot):.1f} us "
          f"({GF / (sum(tot) / len(tot)) * 1e3:.0f} TF/s){ev}")


if __name__ == "__main__":
    main()
