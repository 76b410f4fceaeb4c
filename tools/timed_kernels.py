"""The timed rollout's own launches in a rocprofv3 kernel trace of `bench.py`.

bench.py's dispatch order: GPU warm-up rollouts, the W warmup steps, the TIMED rollout, the stamped
re-run of the timed rollout, then the launch-by-launch replay.  Every rollout call chain starts with
one `gnca_ks_images` launch (the weight images), so the timed rollout is exactly the dispatches from
the second-to-last `gnca_ks_images` up to (excluding) the last one.  Summarised per kernel: launches,
mean / min / max duration, and the segment's device span per step (first start .. last end), next to
the bench line's ms_per_step and its stamp-based K1 duration.

  python tools/timed_kernels.py <run_kernel_trace.csv> <bench.json> [out.json]
"""
import csv
import json
import re
import sys


def kclass(name):
    if "gnca_k1_split" in name:
        return "K1F" if re.search(r", (true|1|2)>", name) else "K1"
    for k in ("gnca_k2_finalize", "gnca_ks_images", "gnca_k_alive", "gnca_k0"):
        if k in name:
            return k
    return name[:40]


def union_ms(rows):
    """Length (ms) of the union of the rows' [start, end] intervals: with the sub-batch pipeline a
    K1 dispatch begins when its first workgroup lands on a CU the other sub-batch's K1 has freed,
    so one launch's begin..end includes time queued behind the other; the union is the time any K1
    was running, the quantity the stamps measure."""
    tot, cur = 0, None
    for s, e in sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows):
        if cur is None or s > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    return (tot + (cur[1] - cur[0] if cur else 0)) / 1e6


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    line = None
    for ln in open(bench):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Dispatch_Id"]))
    img = [i for i, r in enumerate(rows) if "gnca_ks_images" in r["Kernel_Name"]]
    if len(img) < 2:
        raise SystemExit("fewer than two rollout chains in the trace")
    seg = rows[img[-2]:img[-1]]
    steps = line["steps"] if line else None
    per = {}
    for r in seg:
        k = kclass(r["Kernel_Name"])
        per.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    t0 = min(int(r["Start_Timestamp"]) for r in seg)
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:])]
    res = {"source": trace, "dispatch_range": [int(seg[0]["Dispatch_Id"]), int(seg[-1]["Dispatch_Id"])],
           "kernels": {k: {"launches": len(v), "mean_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v),
                           "total_ms": sum(v)} for k, v in per.items()},
           "device_span_ms": (t1 - t0) / 1e6,
           "launch_gap_us": {"mean": sum(gaps) / max(1, len(gaps)), "max": max(gaps, default=0.0)}}
    if line:
        r = line["roofline"]
        res["bench"] = {"ms_per_step": line["ms_per_step"], "steps": steps, "k1_ms_stamps": r["k1_ms"],
                        "kernel": r["kernel"]}
        res["device_span_ms_per_step"] = (t1 - t0) / 1e6 / steps
        k1n = "K1F" if "K1F" in res["kernels"] else "K1"
        k1rows = [x for x in seg if kclass(x["Kernel_Name"]) == k1n]
        k2rows = [x for x in seg if kclass(x["Kernel_Name"]) == "gnca_k2_finalize"]
        if k1rows:
            res["k1_union_ms_per_step"] = union_ms(k1rows) / steps
            res["k2_union_ms_per_step"] = union_ms(k2rows) / steps if k2rows else 0.0
            res["k1_k2_union_ms_per_step"] = union_ms(k1rows + k2rows) / steps
            res["k1_union_over_stamps"] = res["k1_union_ms_per_step"] / r["k1_ms"]
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
