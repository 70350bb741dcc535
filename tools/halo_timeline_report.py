"""Report of a halo-conv phase timeline captured by tools/halo_timeline.py (host-side).

usage: python tools/halo_timeline_report.py gpurun_out/ht_fwd.npy
Cycles are s_memtime ticks (shader clock).  Per workgroup: prologue (start -> first barrier), the 20 main-loop
steps, epilogue (loop end -> end); per CU: how many workgroups overlap and the idle gaps between them.
"""
import collections
import sys

import numpy as np

t = np.load(sys.argv[1]).astype(np.int64)          # [nwg][2 waves][32]
hw, xcc = t[:, 0, 0], t[:, 0, 1]
cu = ((xcc & 15) << 12) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
for w in range(2):
    ts = t[:, w]
    start, pro, end, lend = ts[:, 2], ts[:, 3], ts[:, 31], ts[:, 30]
    steps = np.diff(ts[:, 3:24], axis=1)           # 20 steps
    print(f"wave {w * 4}: lifetime {np.median(end - start):8.0f}  prologue {np.median(pro - start):7.0f}  "
          f"loop {np.median(lend - pro):8.0f}  epilogue {np.median(end - lend):7.0f}  (median ticks)")
    ph = lambda a, b: np.median(ts[:, b] - ts[:, a])
    print(f"   prologue: tables {ph(2, 24):.0f}, table barrier {ph(24, 25):.0f} (+first loads issued), "
          f"first-halo transform+store {ph(25, 26):.0f}, first barrier {ph(26, 3):.0f}")
    print(f"   epilogue: pack+stats {ph(30, 27):.0f}, barrier {ph(27, 28):.0f}, stores {ph(28, 31):.0f}")
    print("   per-step median:", " ".join(f"{v:.0f}" for v in np.median(steps, axis=0)))
    print("   per-step p90   :", " ".join(f"{v:.0f}" for v in np.percentile(steps, 90, axis=0)))
t0 = t[:, :, 2].min()
span = t[:, :, 31].max() - t0
print(f"kernel span {span} ticks; workgroups {len(t)}; CUs seen {len(set(cu.tolist()))}")
per = collections.defaultdict(list)
for i in range(len(t)):
    per[int(cu[i])].append((int(t[i, 0, 2] - t0), int(t[i, 0, 31] - t0)))
conc, gaps, nper = [], [], []
for k, iv in per.items():
    iv.sort()
    nper.append(len(iv))
    ev = sorted([(s, 1) for s, e in iv] + [(e, -1) for s, e in iv])
    c = 0
    last = 0
    acc = collections.Counter()
    for x, d in ev:
        acc[c] += x - last
        c += d
        last = x
    tot = sum(acc.values())
    conc.append({kk: v / tot for kk, v in acc.items()})
print("workgroups per CU:", collections.Counter(nper).most_common(5))
avg = collections.Counter()
for cc in conc:
    for kk, v in cc.items():
        avg[kk] += v / len(conc)
print("fraction of each CU's busy span with k resident workgroups:", {k: round(v, 3) for k, v in sorted(avg.items())})
k0 = sorted(per)[0]
print("example CU timeline (start, end, ticks from kernel start):", per[k0][:12])
