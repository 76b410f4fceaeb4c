"""Summarise tools/pmc.sh output: per kernel, mean of each counter per dispatch."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        # the fold instances: gnca_k1_split's 6th template argument (FOLD) is 1 or 2
        fold = re.search(r"gnca_k1_split<\d+, \d+, \d+, \d+, \d+, ([12])\b", k)
        k = ("K1F" if fold else "K1") if "gnca_k1" in k else ("K2" if "k2_finalize" in k else k.replace("gnca::", "").replace("(anonymous namespace)::", "")[:48])
        vals[k][(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
for k, d in vals.items():
    per = defaultdict(list)
    for (cn, disp), v in d.items():
        per[cn].append(sum(v))
    print(f"== {k}")
    for cn in sorted(per):
        v = per[cn]
        print(f"  {cn:32s} {sum(v)/len(v):16.6g}   (n={len(v)})")
