"""Per-kernel average durations from a rocprofv3 kernel trace of `bench.py` next to the bench
line's own HIP-event averages (roofline k1_ms / k2_ms).  The trace of `bench.py --no-cpu` holds,
per kernel, W warmup launches, then K timed and K replayed launches (bench.py's K1/K2 averages are
over the replayed launches, which repeat the timed ones' work).

  python tools/prof_agree.py <run_kernel_trace.csv> <bench.json> [warmup]
"""
import csv
import json
import sys

trace, bench = sys.argv[1], sys.argv[2]
W = int(sys.argv[3]) if len(sys.argv) > 3 else 8
b = json.load(open(bench))
rows = list(csv.DictReader(open(trace)))
want = {"K1": (b["roofline"]["kernel"].split("<")[0], b["roofline"]["k1_ms"]),
        "K2": ("gnca_k2_finalize", b["roofline_k2"]["k2_ms"])}
for tag, (name, ms) in want.items():
    k = sorted((r for r in rows if name in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in k]
    rest = d[W:]
    print(f"{tag} {name}: rocprof launches {len(d)}, avg all {sum(d) / len(d):.4f} ms, "
          f"avg after the {W} warmup launches {sum(rest) / len(rest):.4f} ms; bench.py HIP events "
          f"{ms:.4f} ms (ratio {sum(rest) / len(rest) / ms:.3f})")
