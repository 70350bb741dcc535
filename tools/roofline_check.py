"""Cross-check bench.py's live roofline timing against the rocprofv3 kernel trace of the same command.

usage: python tools/roofline_check.py gpurun_out/prof/run_kernel_trace.csv [--n 23]
bench.py's conv_roofline() issues 3 warm-up + 20 timed launches of the dominant problem
(conv3x3_halo<false, 2>, 2048 workgroups) after the train and sampler legs, i.e. the last
launches of that kernel in the trace; prints their mean/min duration (us).
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--n", type=int, default=20)
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.trace))
        if "conv3x3_halo<false, 2>" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 2048 * 512]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-a.n:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in last]
print(f"conv3x3_halo<false, 2> (8x256x256x128->128) last {len(d)} launches: mean {sum(d) / len(d):.1f} us, "
      f"min {min(d):.1f} us, max {max(d):.1f} us")
