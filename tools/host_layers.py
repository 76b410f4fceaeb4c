"""Per-step host cost by layer at the trainer's size (dev tool, GPU box): raw C call, step.step(),
module forward (no grad / with autograd).  python tools/host_layers.py"""
import ctypes
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_cellular_automata_amd import NeuralCAGraph, _lib as L, step as S  # noqa: E402
from graph_neural_cellular_automata_amd.modules._stepper import run_step  # noqa: E402

dev = torch.device("cuda:0")
B, H, C, T = 16, 40, 16, 400
torch.manual_seed(0)
random.seed(0)
model = NeuralCAGraph(C, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                      graph_zero_padded_shift=False).to(dev)
x = torch.rand(B, C, H, H, device=dev)
active = torch.ones(B, dtype=torch.bool, device=dev)
lib = L.load()
offs = random.sample(model.graph.offsets, 8)
tensors = dict(perception=model.perception.conv.weight, w1=model.update_net[0].weight, b1=model.update_net[0].bias,
               w2=model.update_net[2].weight, gn_weight=model.norm.weight, gn_bias=model.norm.bias)
tensors.update(model.graph.weight_tensors())
w, keep = S.make_weights(tensors)
d = S.make_desc(B=B, C=C, H=H, W=H, hidden=128, d_model=16, offsets=offs,
                flags=L.USE_GROUPNORM | L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE, update_gain=0.05, alpha_thr=0.12,
                message_gain=0.25, fire_rate=0.7, fire_mode=L.FIRE_HASH)
ws = S.workspace(d, dev)
out = torch.empty_like(x)
act = active.view(torch.uint8)
sp = torch.cuda.current_stream().cuda_stream


def t_it(name, fn):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(T):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:34s} host {1e6 * (t1 - t0) / T:7.1f} us/step   wall {1e6 * (t2 - t0) / T:7.1f} us/step", flush=True)


t_it("raw gnca_step_masked_f32", lambda: lib.gnca_step_masked_f32(ctypes.byref(d), ctypes.byref(w), x.data_ptr(),
                                                                  out.data_ptr(), None, act.data_ptr(), ws.data_ptr(),
                                                                  ws.numel(), sp))
t_it("step.step (masked, hash fire)", lambda: S.step(d, w, x, active=active))
t_it("torch.rand(B,1,H,W)", lambda: torch.rand(B, 1, H, H, device=dev))
with torch.no_grad():
    t_it("module forward, no grad", lambda: model(x, fire_rate=0.7, active=active))
xg = x.clone().requires_grad_(True)
t_it("module forward, autograd", lambda: model(xg, fire_rate=0.7, active=active))
