"""Opcode histogram of the innermost loop of a kernel in a hipcc .s file, where the loop is
taken as the span from its 'Loop Header' label back to the last branch that targets the
header or a label placed just before it (latch blocks the compiler moves above the header).
usage: python scripts/asm_range_stats.py file.s kernel_substring"""
import re
import sys
from collections import Counter

path, kname = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kname in l and ":" in l.split(";")[0])
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
for h, l in enumerate(body):
    if "Loop Header" not in l:
        continue
    label = l.split(":")[0]
    # labels within 25 lines above the header (a rotated latch) also count as the loop
    near = {label} | {body[i].split(":")[0] for i in range(max(0, h - 25), h) if re.match(r"^\.LBB\w+:", body[i])}
    lo = min([h] + [i for i in range(max(0, h - 25), h) if re.match(r"^\.LBB\w+:", body[i])])
    back = max(i for i, x in enumerate(body)
               if any(re.search(r"s_(c?branch)\w*\s+" + re.escape(n) + r"$", x) for n in near))
    c = Counter()
    for x in body[lo:back + 1]:
        t = x.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        c[t.split()[0]] += 1
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
    print(f"loop {label}: lines {lo}-{back}, {sum(c.values())} instr, VALU {valu}, MFMA {mf}")
    for k, v in c.most_common(22):
        print(f"   {v:4d} {k}")
