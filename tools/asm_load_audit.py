"""Audit hand-counted asm register loads in a kernel's gfx950 assembly (host-side helper).

usage: python tools/asm_load_audit.py FILE.s KERNEL_SYMBOL_SUBSTRING
hipcc treats an inline-asm load's destination as written at ;;#ASMEND, so it may copy, spill or reuse the register
before the data lands.  This walks the kernel text in order, tracks every VMEM op (asm loads, asm LDS-DMA, and
compiler VMEM ops), retires them at each s_waitcnt vmcnt(N) (all but the newest N), and reports any non-asm
instruction that touches the destination VGPRs of a still-pending asm load.  Text order approximates execution
order: straight-line code with branches only around whole phases.
"""
import re
import sys

src = open(sys.argv[1]).read()
key = sys.argv[2]
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", src, re.M) if key in m.group(1)]
for name in names:
    i = src.index(name + ":")
    j = src.index(".Lfunc_end", i)
    lines = src[i:j].split("\n")
    in_asm = False
    pend = []   # list of (kind, set of vgprs)
    bad = []
    nload = 0

    def regs(text):
        out = set()
        for m in re.finditer(r"\bv\[(\d+):(\d+)\]", text):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        for m in re.finditer(r"\bv(\d+)\b", text):
            out.add(int(m.group(1)))
        return out

    for ln, l in enumerate(lines):
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        m = re.search(r"vmcnt\((\d+)\)", t)
        if op == "s_waitcnt" and m:
            keep = int(m.group(1))
            pend = pend[len(pend) - keep:] if keep < len(pend) else pend
            if keep == 0:
                pend = []
            continue
        is_vmem = op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load", "global_store",
                                 "scratch_store", "buffer_store", "global_atomic"))
        if in_asm and op.startswith("global_load_dwordx4"):
            dst = t.split()[1].rstrip(",")
            pend.append(("asm", regs(dst)))
            nload += 1
            continue
        if in_asm and op.startswith("global_load_lds"):
            pend.append(("dma", set()))
            continue
        if in_asm:
            continue
        touched = regs(t)
        for kind, rs in pend:
            if kind == "asm" and rs & touched:
                bad.append((ln, t))
                break
        if is_vmem and op.startswith(("global_load", "scratch_load", "buffer_load", "flat_load")):
            pend.append(("cc", set()))
    print(f"{name[:70]}: {nload} asm loads, {len(bad)} touches of pending asm-load registers")
    for ln, t in bad[:12]:
        print(f"   line {ln}: {t}")
