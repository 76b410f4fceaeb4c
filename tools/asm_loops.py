"""Per-basic-block instruction mix of one kernel in a hipcc -S output (dev tool)."""
import re
import sys
from collections import Counter

path, kern = sys.argv[1], sys.argv[2]
s = open(path).read()
i = s.index(kern + ":")
j = s.index(".Lfunc_end", i)
blocks, cur, name = [], [], "entry"
for line in s[i:j].split("\n")[1:]:
    m = re.match(r"^(\.LBB\d+_\d+):", line)
    if m:
        blocks.append((name, cur)); name, cur = m.group(1), []
        continue
    t = line.strip()
    if not t or t.startswith((";", ".")):
        continue
    cur.append(t.split()[0])
blocks.append((name, cur))
for name, ops in blocks:
    c = Counter(ops)
    tot = len(ops)
    if tot < 15 and not (c.get("v_mfma_f32_16x16x4_f32") or c.get("v_mfma_f32_32x32x16_bf16")):
        continue
    mf = c.get("v_mfma_f32_16x16x4_f32", 0) + c.get("v_mfma_f32_32x32x16_bf16", 0)
    ds = sum(v for k, v in c.items() if k.startswith("ds_"))
    vm = sum(v for k, v in c.items() if k.startswith(("global_", "flat_", "buffer_")))
    sa = sum(v for k, v in c.items() if k.startswith("s_"))
    rl = c.get("v_readlane_b32", 0) + c.get("v_writelane_b32", 0)
    br = [o for o in ops if o.startswith("s_cbranch") or o == "s_branch"]
    print(f"{name:14s} n={tot:5d} mfma={mf:4d} ds={ds:4d} vmem={vm:3d} salu={sa:4d} lane={rl:3d} waitcnt={c.get('s_waitcnt',0):4d} nop={c.get('s_nop',0):3d}")
