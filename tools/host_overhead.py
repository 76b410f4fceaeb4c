"""Host-side cost of the per-step module API at the trainer's size (dev tool, GPU box):
wall time of a 200-step rollout (no_grad / with autograd graph) and of its backward, against the
GPU time of the same launches (HIP events).  python tools/host_overhead.py"""
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_cellular_automata_amd import NeuralCAGraph  # noqa: E402

dev = torch.device("cuda:0")
B, H, C, T = 16, 40, 16, 200
torch.manual_seed(0)
random.seed(0)
model = NeuralCAGraph(C, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                      graph_zero_padded_shift=False).to(dev)
with torch.no_grad():
    model.update_net[2].weight.normal_(0, 0.05)
x0 = torch.rand(B, C, H, H, device=dev)
active = torch.ones(B, dtype=torch.bool, device=dev)


def roll(grad):
    x = x0.clone().requires_grad_(grad)
    for t in range(T):
        x = model(x, fire_rate=0.7, active=active)
    return x


for grad in (False, True):
    for rep in range(2):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        with torch.set_grad_enabled(grad):
            x = roll(grad)
        t_issue = time.perf_counter() - t0
        e1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"forward grad={grad}: wall {wall * 1e6 / T:.1f} us/step, host issue {t_issue * 1e6 / T:.1f} "
              f"us/step, GPU span {e0.elapsed_time(e1) * 1e3 / T:.1f} us/step", flush=True)
        if grad:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            x.sum().backward()
            t_issue = time.perf_counter() - t0
            e1.record()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            print(f"backward: wall {wall * 1e6 / T:.1f} us/step, host issue {t_issue * 1e6 / T:.1f} us/step, "
                  f"GPU span {e0.elapsed_time(e1) * 1e3 / T:.1f} us/step", flush=True)
            model.zero_grad(set_to_none=True)
