"""Per-basic-block mix of one kernel in a `hipcc -S` listing, with loop nesting (dev tool).
usage: python tools/asm_blocks.py file.s <mangled-kernel-name-substring>"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = re.findall(r"^(_Z\w+):", s, re.M)
kern = [n for n in names if sys.argv[2] in n][0]
i = s.index(kern + ":")
j = s.index(".Lfunc_end", i)
blocks, cur, name, info = [], [], "entry", ""
for line in s[i:j].split("\n")[1:]:
    m = re.match(r"^(\.LBB\d+_\d+):(.*)", line)
    if m:
        blocks.append((name, info, cur)); name, info, cur = m.group(1), m.group(2).strip(), []
        continue
    t = line.strip()
    if t and not t.startswith((";", ".")):
        cur.append(t.split()[0])
blocks.append((name, info, cur))
print(kern)
tot = Counter()
for name, info, ops in blocks:
    c = Counter()
    for o in ops:
        if o.startswith("v_mfma"): c["mfma"] += 1
        elif o.startswith("v_"): c["valu"] += 1
        elif o.startswith("ds_"): c["lds"] += 1
        elif o.startswith(("global_", "buffer_", "scratch_", "flat_")): c["vmem"] += 1
        elif o.startswith("s_nop"): c["nop"] += 1
        elif o.startswith("s_"): c["salu"] += 1
    depth = re.search(r"Depth=(\d+)", info)
    d = int(depth.group(1)) if depth else 0
    print(f"{name:12s} d={d} " + " ".join(f"{k}={c[k]}" for k in ("valu", "mfma", "lds", "vmem", "salu", "nop")))
