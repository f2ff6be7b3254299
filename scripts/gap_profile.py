"""Per-MFMA-gap instruction mix of the main loop of a kernel in a hipcc .s file: for each MFMA
in the largest loop block, the instructions issued between it and the next MFMA, with a rough
issue-cycle estimate (MI355X_MICROARCH.md 'vector-instruction ISSUE cost').
usage: python scripts/gap_profile.py file.s mangled_kernel_name"""
import re
import sys

path, kname = sys.argv[1], sys.argv[2]
L = open(path).read().split("\n")
a = next(i for i, l in enumerate(L) if l.startswith(kname + ":"))
b = next(i for i in range(a, len(L)) if L[i].startswith(".Lfunc_end"))
L = L[a:b]
# blocks
blocks, cur = [], []
for l in L:
    if re.match(r"^(\.LBB\w+|; %bb\.\d+):", l):
        blocks.append(cur)
        cur = []
    t = l.strip()
    if t and not t.startswith(";") and not t.startswith(".") and not t.endswith(":"):
        cur.append(t.split()[0])
blocks.append(cur)
body = max(blocks, key=lambda blk: sum(1 for x in blk if x.startswith("v_mfma")))
cost = lambda op: (8 if op.startswith("v_mfma") else 8 if op.startswith("v_exp") else 4 if op.startswith("v_") else
                   4 if op.startswith("ds_") else 4 if op == "s_nop" else 1)
gaps, g = [], None
for op in body:
    if op.startswith("v_mfma"):
        if g is not None:
            gaps.append(g)
        g = [op]
    elif g is not None:
        g.append(op)
if g:
    gaps.append(g)
tot = 0
for i, g in enumerate(gaps):
    c = sum(cost(op) for op in g)
    tot += max(c, 32)
    kinds = {}
    for op in g[1:]:
        k = "exp" if op.startswith("v_exp") else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else \
            "wait" if op == "s_waitcnt" else "nop" if op == "s_nop" else "vmem" if op.startswith("buffer") else "salu"
        kinds[k] = kinds.get(k, 0) + 1
    print(f"gap {i:2d}: ~{c:3d} cyc  " + " ".join(f"{k}={v}" for k, v in sorted(kinds.items())))
print(f"{len(gaps)} gaps, sum of max(issue, 32) = {tot} cycles")
