"""cProfile of the per-step module forward with autograd (dev tool, GPU box)."""
import cProfile
import os
import pstats
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_cellular_automata_amd import NeuralCAGraph  # noqa: E402

dev = torch.device("cuda:0")
B, H, C, T = 16, 40, 16, 300
torch.manual_seed(0)
random.seed(0)
model = NeuralCAGraph(C, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                      graph_zero_padded_shift=False).to(dev)
x0 = torch.rand(B, C, H, H, device=dev)
active = torch.ones(B, dtype=torch.bool, device=dev)


def roll():
    x = x0.clone().requires_grad_(True)
    for t in range(T):
        x = model(x, fire_rate=0.7, active=active)
    return x


roll()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
x = roll()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
