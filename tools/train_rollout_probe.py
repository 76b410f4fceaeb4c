"""Host vs GPU time of the graph trainer's BPTT rollout loop at the trainer's size (dev tool, GPU
box): the bench's loop body (masked steps, fire ~ U(0.5,0.9), message every 3rd step), variants
switched off one at a time.  python tools/train_rollout_probe.py"""
import gc
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
x0 = torch.zeros(B, C, H, H, device=dev)
x0[:, 3, H // 2, H // 2] = 1.0
nsteps = torch.randint(150, 201, (B,), device=dev)


def loop(toggle_msg, rand_fire, mask, grad=True):
    x = x0.clone()
    for t in range(T):
        fr = random.uniform(0.5, 0.9) if rand_fire else 0.7
        if toggle_msg:
            model.message_gain = 0.25 if t % 3 == 0 else 0.0
        x = model(x, fire_rate=fr, active=(nsteps > t) if mask else None)
    model.message_gain = 0.25
    return x


BENCH = dict(toggle_msg=True, rand_fire=True, mask=True)
for name, kw, nogc in (("bench loop", BENCH, False), ("no message toggle", dict(BENCH, toggle_msg=False), False),
                       ("no mask", dict(BENCH, mask=False), False), ("bench loop", BENCH, False),
                       ("bench loop, gc off", BENCH, True), ("bench loop", BENCH, False)):
    if nogc:
        gc.disable()
    for rep in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        x = loop(**kw)
        e1.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        l = x[:, :4].square().mean()
        t3 = time.perf_counter()
        l.backward()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"{name:20s} fwd: host {1e6 * (t1 - t0) / T:6.1f} us/step, wall {1e6 * (t2 - t0) / T:6.1f}, "
              f"GPU {1e3 * e0.elapsed_time(e1) / T:6.1f};  bwd wall {1e6 * (t4 - t3) / T:6.1f} us/step", flush=True)
        model.zero_grad(set_to_none=True)
    gc.enable()
