"""Debug: compare gnca_rollout_f32 with a launch-by-launch replay through gnca_step_phases_f32."""
import ctypes, random, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
from graph_neural_cellular_automata_amd import _lib as L, step as S
from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
dev = torch.device("cuda:0")
lib = L.load()
wl = bench.WORKLOADS["headline"]
B, H, C, K = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 72, 16, 8
tab = GraphAugmentation._build_offsets(4)
w, keep = bench.weight_struct(bench.load_weights(dev, wl), wl)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.rand(B, C, H, H, device=dev, generator=g)
x[:, 4:] = torch.randn(B, C - 4, H, H, device=dev, generator=g)
d0 = bench.make_desc(wl, B, H, H, tab[:K], 0)
ws = S.workspace(d0, dev)
sp = torch.cuda.current_stream().cuda_stream
rr = random.Random(3)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
TORCH_OPS = len(sys.argv) > 3
offs = [rr.sample(tab, K) for _ in range(n)]
flat = [v for o in offs for p in o for v in p]
arr = (ctypes.c_int8 * len(flat))(*flat)
out, scr = torch.empty_like(x), torch.empty_like(x)
L.check(lib.gnca_rollout_f32(ctypes.byref(bench.make_desc(wl, B, H, H, tab[:K], 0, 5)), ctypes.byref(w), n, arr,
                             x.data_ptr(), out.data_ptr(), scr.data_ptr(), ws.data_ptr(), ws.numel(), sp), "roll")
for mode in ("phases", "step"):
    bufs = [torch.empty_like(x), torch.empty_like(x)]
    src = x
    for t in range(n):
        d = bench.make_desc(wl, B, H, H, offs[t], 0, 5 + t)
        dst = bufs[t % 2]
        if TORCH_OPS:
            kp = ((torch.nn.functional.max_pool2d(src[:, 3:4], 3, 1, 1) > 0.12) & (S.fire_mask(d, dev) != 0))[:, 0]
            kk = kp.sum()
        if mode == "phases":
            L.check(lib.gnca_step_phases_f32(ctypes.byref(d), ctypes.byref(w), src.data_ptr(), dst.data_ptr(), None, None,
                                             ws.data_ptr(), ws.numel(), sp, L.PHASE_K1 | (L.PHASE_ALIVE if t else 0)), "k1")
            L.check(lib.gnca_step_phases_f32(ctypes.byref(d), ctypes.byref(w), src.data_ptr(), dst.data_ptr(), None, None,
                                             ws.data_ptr(), ws.numel(), sp, L.PHASE_K2 | L.PHASE_ALIVE), "k2")
        else:
            L.check(lib.gnca_step_phases_f32(ctypes.byref(d), ctypes.byref(w), src.data_ptr(), dst.data_ptr(), None, None,
                                             ws.data_ptr(), ws.numel(), sp, L.PHASE_ALL), "all")
        src = dst
    torch.cuda.synchronize()
    print(mode, "equal" if torch.equal(src, out) else f"DIFF max {float((src - out).abs().max()):.3e}")
