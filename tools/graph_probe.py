"""Probe (measurement only): does capturing a small-batch rollout into a HIP graph shrink the
per-step time?  Times gnca_rollout_f32 (40 steps, fixed offsets) issued directly vs replayed from a
torch.cuda.CUDAGraph capture of the same call.  usage: python tools/graph_probe.py [config]"""
import ctypes
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from graph_neural_cellular_automata_amd import _lib as L  # noqa: E402
from graph_neural_cellular_automata_amd import step as S  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
wl = bench.WORKLOADS[cfg]
dev = torch.device("cuda:0")
lib = L.load()
B, C, H, K = wl["B"], wl["C"], wl["H"], wl["K"]
w, keep = bench.weight_struct(bench.load_weights(dev, wl), wl)
x = torch.rand(B, C, H, H, device=dev)
x[:, 4:] = torch.randn(B, C - 4, H, H, device=dev)
out, scratch = torch.empty_like(x), torch.empty_like(x)
from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
table = GraphAugmentation._build_offsets(wl["R"]) if wl["graph"] else []
n = 40
rr = random.Random(1)
flat = [v for _ in range(n) for o in (rr.sample(table, K) if wl["graph"] else []) for v in o]
arr = (ctypes.c_int8 * max(1, len(flat)))(*flat)
d = bench.make_desc(wl, B, H, H, table[:K], 0)
ws = S.workspace(d, dev)
s = torch.cuda.Stream(dev)


def call():
    L.check(lib.gnca_rollout_f32(ctypes.byref(d), ctypes.byref(w), n, arr if flat else None, x.data_ptr(),
                                 out.data_ptr(), scratch.data_ptr(), ws.data_ptr(), ws.numel(),
                                 torch.cuda.current_stream(dev).cuda_stream), "rollout")


with torch.cuda.stream(s):
    for _ in range(30):
        call()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        call()
    torch.cuda.synchronize()
    ref = out.clone()
    for mode in ("direct", "graph", "direct", "graph"):
        ts = []
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            (g.replay() if mode == "graph" else call())
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3 / n)
        ts.sort()
        assert torch.equal(out, ref)
        print(f"{cfg} {mode:7s} median {ts[len(ts) // 2] * 1e3:.2f} us/step  min {ts[0] * 1e3:.2f}")
