"""cProfile of the module rollout with autograd at the trainer's size (dev tool, GPU box): where the
per-step host time goes.  python tools/host_cprof.py"""
import cProfile
import os
import pstats
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_cellular_automata_amd import NeuralCAGraph  # noqa: E402

dev = torch.device("cuda:0")
B, H, C, T = 16, 40, 16, 400
torch.manual_seed(0)
random.seed(0)
model = NeuralCAGraph(C, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                      graph_zero_padded_shift=False).to(dev)
x0 = torch.rand(B, C, H, H, device=dev)
nsteps = torch.randint(48, 81, (B,), device=dev)


def roll():
    x = x0.clone()
    for t in range(T):
        x = model(x, fire_rate=random.uniform(0.5, 0.9), active=nsteps > t)
    return x


for _ in range(2):
    roll().sum().backward()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
x = roll()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
