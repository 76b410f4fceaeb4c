"""tools/pmc.sh output -> profiles/<round>_pmc_traffic.json (per-launch HBM traffic of K1/K2).

traffic = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes).  The x2 is the gfx950 correction: FETCH_SIZE
reports exactly half the bytes for every load form these kernels use (LDS-DMA dword, dwordx4 and
dword streams; calibrated by tools/ubench/fetch_calib.hip, MI355X_MICROARCH.md §HBM).  Counter rows
of one dispatch (one per XCD / instance) are summed, then averaged over dispatches.

  python tools/pmc_traffic.py [gpurun_out/pmc] [profiles/r01_pmc_traffic.json]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/r01_pmc_traffic.json"
vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        # the fold instances: gnca_k1_split's 6th template argument (FOLD) is 1 or 2
        fold = re.search(r"gnca_k1_split<\d+, \d+, \d+, \d+, \d+, ([12])\b", k)
        k = ("K1F" if fold else "K1") if "gnca_k1" in k else ("K2" if "k2_finalize" in k else None)
        if k:
            vals[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
res = {"fetch_correction": 2.0,
       # rollout launches of each kernel per CA step when the passes ran (2: the sub-batch pipeline)
       "launches_per_step": int(os.environ.get("PMC_LAUNCHES_PER_STEP", "1")),
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                 "`python3 bench.py --steps 4 --warmup 1 --no-cpu` (tools/pmc.sh); "
                 "FETCH_SIZE x2 per tools/ubench/fetch_calib.hip",
       # sha256[:16] of the libgnca.so the passes ran (set by the session script), so that a bench line
       # can tell whether these counters belong to the build it timed
       "lib_sha16": os.environ.get("GNCA_LIB_SHA16"),
       "bench_args": os.environ.get("PMC_CMD") or os.environ.get("BENCH_ARGS"),
       "kernels": {}}
for k, d in vals.items():
    m = {c: sum(v.values()) / len(v) for c, v in d.items()}
    fetch = m.get("FETCH_SIZE", 0.0) * 1024 * 2.0
    write = m.get("WRITE_SIZE", 0.0) * 1024
    res["kernels"][k] = {"hbm_read_bytes": fetch, "hbm_write_bytes": write,
                         "traffic_bytes": fetch + write,
                         "grbm_gui_active_per_xcd": m.get("GRBM_GUI_ACTIVE", 0.0) / 8, "counters": m}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v["traffic_bytes"] for k, v in res["kernels"].items()}))
