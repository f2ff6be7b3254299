"""Count instructions per opcode inside the innermost loop(s) of a kernel in a hipcc .s file.
usage: python scripts/asm_loop_stats.py file.s kernel_substring"""
import re
import sys
from collections import Counter

path, kname = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kname in l and ":" in l)
end = next(i for i in range(start, len(lines)) if ".end_amdhsa_kernel" in lines[i] or lines[i].startswith("\t.size"))
body = lines[start:end]
headers = [i for i, l in enumerate(body) if "Loop Header" in l]
for h in headers:
    label = body[h].split(":")[0]
    # last branch back to this label
    back = max(i for i, l in enumerate(body) if re.search(r"s_cbranch_\w+\s+" + re.escape(label) + r"$", l)
               or re.search(r"s_branch\s+" + re.escape(label) + r"$", l))
    c = Counter()
    for l in body[h:back + 1]:
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        c[t.split()[0]] += 1
    tot = sum(c.values())
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    print(f"loop {label}: {back - h} lines, {tot} instr, VALU {valu}, MFMA {c['v_mfma_f32_32x32x16_bf16']}")
    for k, v in c.most_common(25):
        print(f"   {v:4d} {k}")
