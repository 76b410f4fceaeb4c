"""Phase timers of the headline K1 inside a rollout (measurement tool, GPU box): a -DGNCA_PROFILE
build of the library (GNCA_LIB_PATH) runs the headline rollout (B=1024 72^2 graph torus r=4 K=8)
and gnca_prof_dump returns, per workgroup of the LAST K1 launch, waves 0 and 3's s_memtime cycles
per phase of gnca_k1_split (PROF_MARK ids).  Run once with a two-stream build and once with a
-DGNCA_ROLLOUT_SUBS=1 build to see what the co-resident K2 costs each phase.

  GNCA_LIB_PATH=build_ab/lib_prof.so python tools/pipe_prof.py [steps]
"""
import ctypes
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from graph_neural_cellular_automata_amd import _lib as L  # noqa: E402
from graph_neural_cellular_automata_amd import step as S  # noqa: E402

NAMES = ["dma_issue+wait", "prologue_wait", "gather+perc+split", "preparer", "mfma+epi+zero",
         "tile_bins", "tile_barrier", "loop_top"]


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS["headline"]
    B, H, K = wl["B"], wl["H"], wl["K"]
    w, keep = bench.weight_struct(bench.load_weights(dev, wl), wl)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.rand(B, 16, H, H, device=dev, generator=g)
    x[:, 4:] = torch.randn(B, 12, H, H, device=dev, generator=g)
    from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
    table = GraphAugmentation._build_offsets(wl["R"])
    rr = random.Random(3)
    offs = [rr.sample(table, K) for _ in range(T)]
    d = bench.make_desc(wl, B, H, H, offs[0], 0)
    for _ in range(2):
        S.rollout(d, w, x, T, offs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    S.rollout(d, w, x, T, offs)
    e1.record()
    torch.cuda.synchronize()
    lib = L.load()
    buf = (ctypes.c_ulonglong * (1024 * 16))()
    assert lib.gnca_prof_dump(buf) == 0
    full = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.float64)
    used = full[:, :8].sum(1) > 0
    print(f"lib {os.path.basename(L.LIB_PATH)}: sub-batches {S.rollout_subs(d)}, {T} steps "
          f"{e0.elapsed_time(e1) / T:.4f} ms/step; last K1 launch, {int(used.sum())} workgroups, "
          f"mean kcycles per workgroup (s_memtime)")
    for title, a in (("wave 0", full[used, :8]), ("wave 3 (preparer)", full[used, 8:])):
        tot = a.sum(1).mean()
        print(f"  {title}: total {tot / 1e3:.1f}")
        for i, n in enumerate(NAMES):
            print(f"    {n:22s} {a[:, i].mean() / 1e3:9.1f}  {a[:, i].mean() / tot:6.1%}")


if __name__ == "__main__":
    main()
