"""BB phase profile (measurement tool, not a test): build libgnca with -DGNCA_PROFILE into
build_ablate/, run one backward through it and print the mean s_memtime cycles per workgroup
per phase of gnca_b_mlp.

  python tools/bprof.py build            # in the build container (hipcc)
  python tools/bprof.py run [BxS ...]    # on the GPU box
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build_ab")   # (travels to the GPU box; build_ablate is gpurun-ignored)
LIB = os.path.join(OUT, "libgnca_prof.so")
NAMES = ["weights", "dma_issue", "dma_wait", "planes+compaction", "groups", "epilogue", "fire", "loop_tail"]


def build():
    os.makedirs(OUT, exist_ok=True)
    csrc = os.path.join(ROOT, "graph_neural_cellular_automata_amd", "csrc")
    srcs = [os.path.join(csrc, f) for f in ("gnca_step.hip", "gnca_bwd.hip", "gnca_aux.hip")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-shared", "-DGNCA_PROFILE", "-fno-slp-vectorize", f"-I{ROOT}/include", f"-I{csrc}", *srcs, "-o", LIB])


def run(sizes):
    import random
    import numpy as np
    import torch
    from graph_neural_cellular_automata_amd import _lib as L
    lib = L.load(LIB)   # every op below now runs the profile build
    lib.gnca_bprof_dump.restype = ctypes.c_int
    from graph_neural_cellular_automata_amd import step as S
    from graph_neural_cellular_automata_amd.modules import NeuralCAGraph
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = NeuralCAGraph(16, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                          graph_zero_padded_shift=False).to(dev)
    with torch.no_grad():
        model.update_net[2].weight.normal_(0, 0.05)
    tensors = dict(perception=model.perception.conv.weight, w1=model.update_net[0].weight,
                   b1=model.update_net[0].bias, w2=model.update_net[2].weight,
                   gn_weight=model.norm.weight, gn_bias=model.norm.bias)
    tensors.update(model.graph.weight_tensors())
    w, keep = S.make_weights(tensors)
    want = {n: p for n, p in model.named_parameters() if n in S.GRAD_FIELDS}
    random.seed(1)
    chosen = random.sample(model.graph.offsets, 8)
    flags = L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE
    for spec in sizes:
        B, H = (int(v) for v in spec.split("x"))
        for msg in (0.25, 0.0):
            x = torch.rand(B, 16, H, H, device=dev)
            x[:, 4:] = torch.randn(B, 12, H, H, device=dev)
            gy = torch.randn_like(x)
            d = S.make_desc(B=B, C=16, H=H, W=H, hidden=128, d_model=16, offsets=chosen, flags=flags,
                            update_gain=0.05, alpha_thr=0.12, message_gain=msg, fire_rate=0.5,
                            fire_mode=L.FIRE_HASH, rng_seed=3)
            for _ in range(3):
                S.step_backward(d, w, x, gy, want=want)
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * (1024 * 8))()
            assert lib.gnca_bprof_dump(buf) == 0
            a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.float64)
            a = a[a.sum(1) > 0]
            tot = a.sum(1).mean()
            print(f"B={B} {H}x{H} message_gain={msg}: mean cycles per BB workgroup {tot:.0f} over {len(a)} WGs "
                  f"(max {a.sum(1).max():.0f})")
            for i, nm in enumerate(NAMES):
                if nm != "-":
                    print(f"  {nm:18s} {a[:, i].mean():10.0f} cycles  {100 * a[:, i].mean() / tot:5.1f} %")


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run(sys.argv[2:] or ["16x40"])
