"""Phase timers of the rollout's K1 launches (measurement tool, not a test): the plain K1 (a one-step
rollout) and the fold K1 (the last K1 of a three-step rollout) of the bench workload, from a
-DGNCA_PROFILE build (s_memtime cycles per phase, summed over each workgroup's tiles; waves 0 and 3).

  python tools/fold_prof.py build     # in the build container (hipcc)
  python tools/fold_prof.py run       # on the GPU box
"""
import ctypes
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build_ab")   # (travels to the GPU box; build_ablate is gpurun-ignored)
LIB = os.path.join(OUT, os.environ.get("FOLDPROF_LIB", "lib_foldprof.so"))
EXTRA = os.environ.get("FOLDPROF_DEFS", "").split()   # build: extra -D flags (timing-only ablations)
FNAMES = ["fin: wait preparer", "fin: item loads + xsd wait", "fin: compute + stores", "fin: items",
          "prep: load issue", "prep: stats + constants", "prep: alpha rows", "prep: pooling", "prep: sender plane",
          "prep: keep + list + tables"]
NAMES = ["stage(dma|finalize)", "prologue_wait", "gather+perc", "preparer", "group_mfma+epi", "partial_bins",
         "barrier_after_groups", "loop_top"]


def build():
    os.makedirs(OUT, exist_ok=True)
    src = [os.path.join(ROOT, "graph_neural_cellular_automata_amd", "csrc", f) for f in
           ("gnca_step.hip", "gnca_bwd.hip", "gnca_aux.hip")]
    objs = []
    for s in src:
        o = os.path.join(ROOT, "build", os.path.basename(s) + "." + os.path.basename(LIB) + ".o")
        extra = ["-fno-slp-vectorize", "-DGNCA_PROFILE", *EXTRA] if s.endswith("gnca_step.hip") else []
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                        *extra, f"-I{ROOT}/include", s, "-o", o], check=True, stderr=subprocess.DEVNULL)
        objs.append(o)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", LIB], check=True)


def run():
    os.environ["GNCA_LIB_PATH"] = LIB
    import numpy as np
    import torch
    import bench
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    lib = L.load(LIB)
    lib.gnca_prof_dump.restype = ctypes.c_int
    lib.gnca_fprof_dump.restype = ctypes.c_int
    lib.gnca_arr_dump.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    wl = bench.WORKLOADS[os.environ.get("FOLDPROF_CONFIG", "headline")]
    B, H = wl["B"], wl["H"]
    w, keep = bench.weight_struct(bench.load_weights(dev, wl), wl)
    g = torch.Generator(device=dev).manual_seed(1234)
    x = torch.rand(B, wl["C"], H, H, device=dev, generator=g)
    x[:, 4:] = torch.randn(B, wl["C"] - 4, H, H, device=dev, generator=g)
    from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
    table = GraphAugmentation._build_offsets(wl["R"]) if wl["graph"] else []
    rr = random.Random(0)
    for steps in (1, 3, 1, 3):
        offs = [rr.sample(table, wl["K"]) if wl["graph"] else [] for _ in range(steps)]
        d = bench.make_desc(wl, B, H, H, offs[0], 0)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        S.rollout(d, w, x, steps, offs)
        e1.record()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (1024 * 16))()
        assert lib.gnca_prof_dump(buf) == 0
        full = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.float64)
        fb = (ctypes.c_ulonglong * (1024 * 32))()
        assert lib.gnca_fprof_dump(fb) == 0
        ff = np.frombuffer(fb, dtype=np.uint64).reshape(1024, 32).astype(np.float64)
        ab = (ctypes.c_ulonglong * (1024 * 16 * 8))()
        assert lib.gnca_arr_dump(ab) == 0
        arr = np.frombuffer(ab, dtype=np.uint64).reshape(1024, 16, 8).astype(np.float64)
        kind = "plain K1 (1-step rollout)" if steps == 1 else "fold K1 (last K1 of a 3-step rollout)"
        print(f"== {kind}: rollout {e0.elapsed_time(e1):.3f} ms (profile build), fold={S.rollout_fold(d)}")
        for title, a in (("wave 0 (SIMD 0)", full[:, :8]), ("wave 3 (preparer)", full[:, 8:])):
            a = a[a.sum(1) > 0]
            tot = a.sum(1).mean()
            print(f" {title}: mean cycles per workgroup {tot:.0f} over {len(a)} WGs")
            for i, nm in enumerate(NAMES):
                print(f"  {nm:22s} {a[:, i].mean():12.0f} cycles  {100 * a[:, i].mean() / tot:5.1f} %")
        used = arr[:, :, 7].sum(1) > 0
        print(" per-wave arrival (cycles from the wave's start, mean over WGs): points = DMA+fire issued, prep done, "
              "finalize done, past prologue barrier, groups done, zero items done (tile 0), past tile-0 barrier, end")
        for wv in range(int(os.environ.get("FOLDPROF_WAVES", "8"))):
            print(f"  wave {wv}: " + " ".join(f"{arr[used, wv, k].mean():7.0f}" for k in range(8)))
        if steps > 1:
            for title, f in (("wave 0", ff[:, :16]), ("wave 3 (preparer)", ff[:, 16:])):
                f = f[f.sum(1) > 0]
                print(f" fold sub-phases, {title} (cycles per workgroup; items = finalize items done):")
                for i, nm in enumerate(FNAMES):
                    print(f"  {nm:26s} {f[:, i].mean():12.0f}")


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
