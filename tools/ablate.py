"""K1 ablation timing (measurement tool, not a test): build libgnca variants with -DGNCA_ABLATE
bits, then time K1 of each on the bench workload in ONE process, interleaved rounds.

  python tools/ablate.py build            # in the build container (hipcc)
  python tools/ablate.py run              # on the GPU box
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build_ablate")
VARIANTS = {
    "full": 0, "no_stage": 1, "no_gather": 2, "no_perceive": 4, "no_mfma": 8, "no_store": 16,
    "no_planes": 32, "mfma_only": 1 | 2 | 4 | 16 | 32, "no_mfma_no_store": 8 | 16,
    "stage_only": 2 | 4 | 8 | 16 | 32,
    "no_fire": 64, "no_zero": 128, "no_reduce": 256,
    "no_prep": 2048, "no_prep_no_stage": 2049, "no_tiles": 512, "no_tiles_no_fill": 512 | 1024, "lds_lite": 4096, "lds_linear": 8192,
    "bare": 2 | 4 | 8 | 16 | 32 | 64 | 128 | 256, "bare_no_stage": 1 | 2 | 4 | 8 | 16 | 32 | 64 | 128 | 256,
}


# experiment builds: ABLATE_EXTRA="name=-DFOO=1 -DBAR;name2=-DBAZ" (each built and timed beside the others)
EXTRA = dict(e.split("=", 1) for e in os.environ.get("ABLATE_EXTRA", "").split(";") if "=" in e)
VARIANTS.update({n: f for n, f in EXTRA.items()})
ONLY = [v for v in os.environ.get("ABLATE_ONLY", "").split(",") if v]   # e.g. "full,prof"
CONFIG = os.environ.get("ABLATE_CONFIG", "headline")                    # a bench.py WORKLOADS key


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "graph_neural_cellular_automata_amd", "csrc", "gnca_step.hip")
    procs = []
    for name, bits in list(VARIANTS.items()) + [("prof", None)]:
        if ONLY and name not in ONLY:
            continue
        flags = (["-DGNCA_PROFILE"] if bits is None else
                 bits.split() if isinstance(bits, str) else [f"-DGNCA_ABLATE={bits}"])
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
               *flags, f"-I{ROOT}/include", src, "-o", os.path.join(OUT, f"lib_{name}.so")]
        procs.append(subprocess.Popen(cmd, stderr=subprocess.DEVNULL))
        if len(procs) >= 4:
            procs.pop(0).wait()
    for p in procs:
        p.wait()


def run(reps=15, rounds=3):
    import random
    import torch
    import bench
    from graph_neural_cellular_automata_amd import _lib as L
    dev = torch.device("cuda:0")
    libs = {}
    for name in VARIANTS:
        if ONLY and name not in ONLY:
            continue
        lib = ctypes.CDLL(os.path.join(OUT, f"lib_{name}.so"))
        lib.gnca_step_phases_f32.restype = ctypes.c_int
        lib.gnca_step_phases_f32.argtypes = [ctypes.POINTER(L.StepDesc), ctypes.POINTER(L.Weights)] + \
            [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32]
        lib.gnca_workspace_bytes.restype = ctypes.c_size_t
        lib.gnca_workspace_bytes.argtypes = [ctypes.POINTER(L.StepDesc)]
        libs[name] = lib
    wl = bench.WORKLOADS[CONFIG]
    B, H = wl["B"], wl["H"]
    w, keep = bench.weight_struct(bench.load_weights(dev, wl), wl)
    x = torch.rand(B, wl["C"], H, H, device=dev)
    out = torch.empty_like(x)
    from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
    build_offsets = GraphAugmentation._build_offsets
    offs = random.Random(0).sample(build_offsets(wl["R"]), wl["K"]) if wl["graph"] else []
    d = bench.make_desc(wl, B, H, H, offs, 0)
    ws = torch.empty(next(iter(libs.values())).gnca_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    # rollout mode (default): K1 reads the alive bytes a primed K2 wrote (GNCA_PHASE_ALIVE)
    ph = int(os.environ.get("ABLATE_PHASES", str(L.PHASE_K1 | L.PHASE_ALIVE | L.PHASE_COMPACT)))
    if ph & L.PHASE_ALIVE:
        assert next(iter(libs.values())).gnca_step_phases_f32(
            ctypes.byref(d), ctypes.byref(w), x.data_ptr(), out.data_ptr(), None, None, ws.data_ptr(),
            ws.numel(), st.cuda_stream, L.PHASE_ALL | L.PHASE_ALIVE | L.PHASE_COMPACT) == 0
    res = {n: [] for n in libs}
    for _ in range(rounds):
        for n, lib in libs.items():
            for r in range(reps + 2):
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                rc = lib.gnca_step_phases_f32(ctypes.byref(d), ctypes.byref(w), x.data_ptr(), out.data_ptr(),
                                              None, None, ws.data_ptr(), ws.numel(), st.cuda_stream, ph)
                e1.record(st)
                assert rc == 0, (n, rc)
                torch.cuda.synchronize()
                if r >= 2:
                    res[n].append(e0.elapsed_time(e1))
    for n, v in res.items():
        v.sort()
        print(f"{n:18s} median {v[len(v)//2]:.3f} ms   min {v[0]:.3f} ms")
    if ONLY and "prof" not in ONLY:
        return
    # phase timers of the profile build (s_memtime cycles summed over each workgroup's tiles)
    pl = ctypes.CDLL(os.path.join(OUT, "lib_prof.so"))
    pl.gnca_step_phases_f32.restype = ctypes.c_int
    pl.gnca_step_phases_f32.argtypes = next(iter(libs.values())).gnca_step_phases_f32.argtypes
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    assert pl.gnca_step_phases_f32(ctypes.byref(d), ctypes.byref(w), x.data_ptr(), out.data_ptr(), None,
                                   None, ws.data_ptr(), ws.numel(), st.cuda_stream, ph) == 0
    e1.record(st)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (1024 * 16))()
    assert pl.gnca_prof_dump(buf) == 0
    import numpy as np
    full = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.float64)
    ws = full[:, 8:].sum() > 0
    if os.environ.get("ABLATE_PROF_SETS") == "w03":   # the split K1: wave 0 and the preparer wave 3
        names = ["dma_issue", "dma_wait+barrier", "gather+perc", "preparer", "group_mfma+epi", "partial_bins",
                 "barrier_after_groups", "loop_top"]
        sets = [("wave 0 (SIMD 0, older)", names, full[:, :8]),
                ("wave 3 (SIMD 3, preparer)", names, full[:, 8:])]
    elif os.environ.get("ABLATE_PROF_SETS") == "w07":   # the 32-channel split K1: wave 0 and the preparer wave 7
        names = ["preparer", "phase0_gather+perc", "phase1_staging", "phase1_gather+perc", "next_stage",
                 "mfma+epi", "partials+barrier", "loop_top"]
        sets = [("wave 0 (SIMD 0, group)", names, full[:, :8]),
                ("wave 7 (preparer / stager)", names, full[:, 8:])]
    elif os.environ.get("ABLATE_PROF_SETS") == "w04":   # the split K1: both waves of SIMD 0
        names = ["dma_issue", "fire+dma_wait", "planes", "compaction", "groups", "reduction",
                 "top_barrier", "loop_tail"]
        sets = [("wave 0 (SIMD 0, older)", names, full[:, :8]),
                ("wave 4 (SIMD 0, younger)", names, full[:, 8:])]
    elif ws:
        sets = [("producer wave 0", ["dma_issue", "fire+dma_wait+pbar", "planes+pbar", "compaction",
                                     "y_compute", "wait_empty", "end_tile_pbar", "end_stream"], full[:, :8]),
                ("consumer wave 4", ["wait_full", "compute", "read+flush", "-", "-", "-", "-", "-"], full[:, 8:])]
    else:
        sets = [("wave 0", ["dma_issue", "fire+dma_wait", "planes", "compaction", "groups", "reduction",
                            "-", "loop_tail"], full[:, :8])]
    print(f"prof build: {e0.elapsed_time(e1):.3f} ms")
    for title, names, a in sets:
        a = a[a.sum(1) > 0]
        tot = a.sum(1).mean()
        print(f" {title}: mean cycles per workgroup {tot:.0f} over {len(a)} WGs")
        for i, nm in enumerate(names):
            if nm != "-":
                print(f"  {nm:20s} {a[:, i].mean():12.0f} cycles  {100 * a[:, i].mean() / tot:5.1f} %")


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
