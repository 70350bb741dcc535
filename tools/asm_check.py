"""Static checks on a HIP kernel's gfx950 assembly (host-side helper).

usage: python tools/asm_check.py csrc/conv_halo.hip conv3x3_halo
Compiles the file to assembly and, for every kernel whose name contains the pattern, reports
VGPR/scratch use and the scratch (spill) and s_waitcnt vmcnt(0) instructions that sit between its
first and last MFMA (i.e. inside the MFMA main loop, where they stall the pipeline).
"""
import os
import re
import subprocess
import sys

src, pat = sys.argv[1], sys.argv[2]
here = os.path.dirname(os.path.abspath(src))
out = "/tmp/_asm_check.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", here, "-I",
                os.path.join(here, "..", "..", "include"), "-S", "--cuda-device-only", src, "-o", out],
               check=True, capture_output=True)
s = open(out).read()
for m in re.finditer(r"^(_Z\S*" + re.escape(pat) + r"\S*):", s, flags=re.M):
    name = m.group(1)
    body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
    mf = [i for i, l in enumerate(body) if "v_mfma" in l]
    if not mf:
        continue
    lo, hi = mf[0], mf[-1]
    spills = [i for i, l in enumerate(body) if "scratch_" in l]
    inloop = [i for i in spills if lo <= i <= hi]
    vm0 = [i for i in range(lo, hi) if re.search(r"s_waitcnt\s+vmcnt\(0\)", body[i])]
    vg = re.search(r"\.vgpr_count:\s*(\d+)", s[m.end():])
    print(f"{name[:70]}: lines {len(body)}, mfma {len(mf)} in [{lo},{hi}], spills {len(spills)} "
          f"(in loop {len(inloop)}), vmcnt(0) in loop {len(vm0)}")
