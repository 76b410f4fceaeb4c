"""Scratch (spill) loads / stores per basic block of one kernel in a `hipcc -S` listing, with loop depth
and each block's MFMA count (dev tool).  usage: python tools/asm_spills.py file.s <kernel-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r"^(_Z\w+):", s, re.M)
kern = [n for n in names if sys.argv[2] in n][0]
i = s.index(kern + ":")
j = s.index(".Lfunc_end", i)
name, depth, st, ld, mf, n = "entry", 0, 0, 0, 0, 0
tot_st = tot_ld = 0
rows = []
for line in s[i:j].split("\n")[1:] + [".LBBend:"]:
    m = re.match(r"^(\.LBB\d+_\d+|\.LBBend):(.*)", line)
    if m:
        rows.append((name, depth, st, ld, mf, n))
        name = m.group(1)
        dm = re.search(r"Depth=(\d+)", m.group(2))
        depth = int(dm.group(1)) if dm else 0
        st = ld = mf = n = 0
        continue
    t = line.strip()
    if not t or t.startswith((";", ".")):
        continue
    n += 1
    op = t.split()[0]
    if op.startswith("scratch_store") or (op.startswith("buffer_store") and "Spill" in t):
        st += 1
    if op.startswith("scratch_load") or (op.startswith("buffer_load") and "Reload" in t):
        ld += 1
    if op.startswith("v_mfma"):
        mf += 1
for r in rows:
    tot_st += r[2]; tot_ld += r[3]
    if r[2] or r[3] or r[4]:
        print("%-12s d=%d spill_st=%d spill_ld=%d mfma=%d insts=%d" % r)
print("total spill stores", tot_st, "reloads", tot_ld)
