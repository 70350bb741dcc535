"""Instruction mix of one kernel's gfx950 assembly, per basic block and in total (host-side helper).

usage: python tools/asm_mix.py FILE.s KERNEL_SYMBOL_SUBSTRING
Prints per basic block: MFMA, other VALU, SALU, LDS, VMEM, scratch counts and the block's loop depth comment.
"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read()
key = sys.argv[2]
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", src, re.M) if key in m.group(1)]
name = names[0]
i = src.index(name + ":")
j = src.index(".Lfunc_end", i)
blocks, cur, label = [], Counter(), "entry"
for line in src[i:j].split("\n"):
    t = line.strip()
    if re.match(r"^\.LBB\S+:", t):
        blocks.append((label, cur))
        cur, label = Counter(), t
        continue
    if not t or t.startswith((";", ".")):
        continue
    op = t.split()[0]
    if op.startswith("v_mfma"):
        cur["mfma"] += 1
    elif op.startswith("v_"):
        cur["valu"] += 1
    elif op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        cur["wait"] += 1
    elif op.startswith("s_"):
        cur["salu"] += 1
    elif op.startswith("ds_"):
        cur["lds"] += 1
    elif op.startswith("scratch_"):
        cur["scratch"] += 1
    elif op.startswith(("global_", "buffer_")):
        cur["vmem"] += 1
blocks.append((label, cur))
tot = Counter()
print(name)
for lab, c in blocks:
    tot.update(c)
    if sum(c.values()) >= 20:
        print(f"{lab[:60]:60s} " + " ".join(f"{k}={c[k]}" for k in ("mfma", "valu", "salu", "lds", "vmem", "scratch", "wait")))
print("total", dict(tot))
