"""Per-MFMA-gap issue estimate of one loop of a kernel in a hipcc .s file: the blocks hipcc
annotates as the loop's header or 'in Loop: Header=<H>', in file order; prints the gaps whose
issue cost (MI355X_MICROARCH.md 'vector-instruction ISSUE cost') exceeds the MFMA's own
pipe time, and the totals.
usage: python scripts/loop_gaps.py file.s mangled_kernel_name BBname [min_cycles]"""
import re
import sys

path, kname, hdr = sys.argv[1], sys.argv[2], sys.argv[3]
thr = int(sys.argv[4]) if len(sys.argv) > 4 else 0
L = open(path).read().split("\n")
a = next(i for i, l in enumerate(L) if l.startswith(kname + ":"))
b = next(i for i in range(a, len(L)) if L[i].startswith(".Lfunc_end"))
ops, inloop = [], False
for l in L[a:b]:
    m = re.match(r"^(\.LBB\w+|; %bb\.\d+):(.*)", l)
    if m:
        inloop = (m.group(1) == "." + "L" + hdr or m.group(1) == ".L" + hdr) or ("Header=" + hdr + " ") in (m.group(2) + " ")
        continue
    t = l.strip()
    if inloop and t and not t.startswith((";", ".")):
        ops.append(t.split()[0])
cost = lambda op: (8 if op.startswith(("v_mfma", "v_exp")) else 4 if op.startswith(("v_", "ds_")) or op == "s_nop" else 1)
pipe = lambda op: 16 if "16x16" in op else 32
gaps, g = [], None
for op in ops:
    if op.startswith("v_mfma"):
        if g is not None:
            gaps.append(g)
        g = [op]
    elif g is not None:
        g.append(op)
if g:
    gaps.append(g)
tot_issue = sum(sum(cost(o) for o in g) for g in gaps)
tot_pipe = sum(pipe(g[0]) for g in gaps)
print(f"{len(ops)} instructions, {len(gaps)} MFMAs: pipe {tot_pipe} cyc, issue {tot_issue} cyc, "
      f"sum of max(issue, pipe) per gap {sum(max(sum(cost(o) for o in g), pipe(g[0])) for g in gaps)} cyc")
for i, g in enumerate(gaps):
    c = sum(cost(o) for o in g)
    if c - pipe(g[0]) > thr:
        kinds = {}
        for op in g[1:]:
            k = ("exp" if op.startswith("v_exp") else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_")
                 else "wait" if op.startswith("s_waitcnt") else "vmem" if op.startswith(("buffer", "global", "scratch"))
                 else "salu")
            kinds[k] = kinds.get(k, 0) + 1
        print(f"  gap {i:3d} after {g[0][7:27]:20s} ~{c:4d} cyc  {kinds}")
