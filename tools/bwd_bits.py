"""Write one backward's outputs (dx and every parameter gradient) at a few sizes to an .npz, so two
library builds (GNCA_LIB_PATH) can be compared bit for bit (dev tool, GPU box):
  GNCA_LIB_PATH=a.so python tools/bwd_bits.py out_a.npz; ... out_b.npz; python tools/bwd_bits.py --cmp a b"""
import os
import random
import sys

import numpy as np

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print("bitwise equal" if not bad and a.files == b.files else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graph_neural_cellular_automata_amd import _lib as L, step as S  # noqa: E402
from graph_neural_cellular_automata_amd.modules import NeuralCAGraph  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for (B, H, zp) in ((16, 40, False), (128, 72, False), (1024, 72, False), (16, 40, True)):
    torch.manual_seed(0)
    model = NeuralCAGraph(16, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                          graph_zero_padded_shift=zp).to(dev)
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
    flags = L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE | (L.ZERO_PAD_SHIFT if zp else 0)
    x = torch.rand(B, 16, H, H, device=dev)
    x[:, 4:] = torch.randn(B, 12, H, H, device=dev)
    gy = torch.randn_like(x)
    d = S.make_desc(B=B, C=16, H=H, W=H, hidden=128, d_model=16, offsets=chosen, flags=flags,
                    update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                    fire_mode=L.FIRE_HASH, rng_seed=3)
    gx, grads = S.step_backward(d, w, x, gy, want=want)
    tag = f"{B}x{H}{'zp' if zp else ''}"
    out[f"{tag}/dx"] = gx.cpu().numpy()
    for k, v in grads.items():
        out[f"{tag}/{k}"] = v.detach().cpu().numpy()
np.savez(sys.argv[1], **out)
print("wrote", sys.argv[1], len(out), "arrays")
