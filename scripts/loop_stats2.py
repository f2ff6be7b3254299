"""Instruction mix of every outermost loop of one kernel in a hipcc .s file: the blocks
hipcc annotates as the loop header or "in Loop: Header=..." of it.
usage: python scripts/loop_stats2.py file.s mangled_kernel_name"""
import collections
import re
import sys

path, kname = sys.argv[1], sys.argv[2]
L = open(path).read().split("\n")
a = next(i for i, l in enumerate(L) if l.startswith(kname + ":"))
b = next(i for i in range(a, len(L)) if L[i].startswith(".Lfunc_end"))
L = L[a:b + 1]
blocks, cur = [], None  # (label line, header of the loop it belongs to)
for i, l in enumerate(L):
    if re.match(r"^(\.LBB\w+|; %bb\.\d+):", l):
        m = re.search(r"Header=(BB\w+)", l)
        hdr = m.group(1) if m else (l.split(":")[0][1:] if "Loop Header" in l else None)
        cur = hdr
        blocks.append((i, hdr))
loops = collections.defaultdict(collections.Counter)
for bi, (i, hdr) in enumerate(blocks):
    if hdr is None:
        continue
    end = blocks[bi + 1][0] if bi + 1 < len(blocks) else len(L)
    for l in L[i + 1:end]:
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        loops[hdr][t.split()[0]] += 1
for hdr, c in loops.items():
    mf = sum(n for k, n in c.items() if k.startswith("v_mfma"))
    valu = sum(n for k, n in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    print(f"{hdr}: {sum(c.values())} instr, VALU {valu}, MFMA {mf}, VALU/MFMA {valu / max(mf, 1):.2f}, "
          f"scratch {sum(n for k, n in c.items() if 'scratch' in k)}, "
          f"moves {c['v_mov_b32_e32'] + c['v_mov_b64_e32']}, readfirstlane {c['v_readfirstlane_b32']}, "
          f"waitcnt {c['s_waitcnt']}, nop {c['s_nop']}")
    for k, n in c.most_common(14):
        print(f"    {n:4d} {k}")
