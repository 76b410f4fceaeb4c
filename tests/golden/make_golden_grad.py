"""Generate the GRADIENT fixtures tests/golden/grad_*.npz by running the REFERENCE's autograd.

Run in the build container only (it needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_grad.py

Two kinds of fixture (data only; the reference source never leaves the container):

* ``grad_<case>``: ONE step.  The input state, the weights, the recorded draws (offsets,
  fire mask), a seeded cotangent ``cot`` for the step output, and the reference's vector-Jacobian
  product ``d(sum(out*cot))`` w.r.t. the state (``gx``) and every parameter that gets a gradient
  (``g:<key>``) — in float32 (the reference's own arithmetic) and float64 (``gx_f64``,
  ``g64:<key>``, the truth the oracle is pinned to).
* ``bptt_<case>``: a short BPTT rollout exactly as the graph trainer runs it
  (``train_graph_augmented_nca.py:302-321``: per-sample step counts, ``state[mask] =
  model(state[mask], fire_rate=fr)``; loss ``loss_premult_rgba`` ``:52-61``, mean over the
  batch), recording every step's offsets / fire mask / fire rate / active mask and the
  reference's gradients.  The fire masks are the sub-batch ``torch.rand`` draws the reference
  made.
"""
from __future__ import annotations

import copy
import json
import os
import random
import sys
import zlib

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import (BASE, CK_CLASSIC, CK_GRAPH, blob_state, grow, load_state,  # noqa: E402
                         make_classic, make_graph, random_state)

OUT = os.path.dirname(os.path.abspath(__file__))


def _draws(model, B, H, W, fire_rate, graph, rng_seed, torch_seed):
    random.seed(rng_seed)
    torch.manual_seed(torch_seed)
    py_state, th_state = random.getstate(), torch.get_rng_state()
    chosen = []
    if graph:
        k = min(model.graph.num_neighbors, len(model.graph.offsets))
        chosen = random.sample(model.graph.offsets, k) if k > 0 else []
    fire = (torch.rand(B, 1, H, W) <= fire_rate) if fire_rate < 1.0 else None
    return chosen, fire, py_state, th_state


def _vjp(model, x, cot, fire_rate, py_state, th_state):
    model.zero_grad(set_to_none=True)
    xl = x.clone().requires_grad_(True)
    random.setstate(py_state)
    torch.set_rng_state(th_state)
    out = model(xl, fire_rate=fire_rate)
    (out * cot).sum().backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    return out.detach(), xl.grad.detach(), grads


def save_grad_case(name, model, knobs, x, fire_rate, *, graph=True, rng_seed=99, torch_seed=77):
    B, C, H, W = x.shape
    chosen, fire, py_state, th_state = _draws(model, B, H, W, fire_rate, graph, rng_seed, torch_seed)
    gen = torch.Generator().manual_seed(zlib.crc32(name.encode()) & 0xFFFF)
    cot = torch.randn(B, C, H, W, generator=gen)
    model = model.train()
    out, gx, grads = _vjp(model, x, cot, fire_rate, py_state, th_state)
    m64 = copy.deepcopy(model).double()
    out64, gx64, grads64 = _vjp(m64, x.double(), cot.double(), fire_rate, py_state, th_state)
    fields = {"w:" + k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    fields.update(x_in=x.numpy(), cot=cot.numpy(), x_out1=out.numpy(), x_out1_f64=out64.numpy(),
                  gx=gx.numpy(), gx_f64=gx64.numpy())
    for k, v in grads.items():
        fields["g:" + k] = v.numpy()
        fields["g64:" + k] = grads64[k].numpy()
    fields["offsets"] = np.array([chosen], dtype=np.int32).reshape(1, len(chosen), 2)
    if fire is not None:
        fields["fire_mask"] = fire.numpy().astype(np.uint8)[None]
    meta = dict(knobs, graph=graph, fire_rate=fire_rate, rng_seed=rng_seed, torch_seed=torch_seed,
                rollout=1, name=name, grad_keys=sorted(grads))
    fields["meta"] = np.array(json.dumps(meta))
    path = os.path.join(OUT, "grad_" + name + ".npz")
    np.savez_compressed(path, **fields)
    print(f"grad_{name}: {os.path.getsize(path)/1024:.0f} KB grads={sorted(grads)}")


def loss_premult_rgba(pred, target):
    """The graph trainer's loss (train_graph_augmented_nca.py:52-61), restated."""
    rgba = torch.cat([pred[:, :3] * pred[:, 3:4], pred[:, 3:4]], dim=1)
    return F.mse_loss(rgba, target, reduction="none").mean(dim=(1, 2, 3))


def _bptt(model, x0, target, steps, frs, use_graph, gain, seed):
    """The trainer's inner loop (train_graph_augmented_nca.py:302-321) with recorded draws."""
    random.seed(seed)
    torch.manual_seed(seed)
    rec = []
    leaf = x0.clone().requires_grad_(True)
    state = leaf * 1.0
    for t in range(int(steps.max())):
        mask = steps > t
        if hasattr(model, "message_gain"):
            model.message_gain = gain if use_graph[t] else 0.0
        py_state, th_state = random.getstate(), torch.get_rng_state()
        nb = int(mask.sum())
        chosen = []
        if hasattr(model, "graph"):
            k = min(model.graph.num_neighbors, len(model.graph.offsets))
            chosen = random.sample(model.graph.offsets, k) if k > 0 else []
        fire = (torch.rand(nb, 1, *x0.shape[2:]) <= frs[t]) if frs[t] < 1.0 else None
        random.setstate(py_state)
        torch.set_rng_state(th_state)
        state[mask] = model(state[mask], fire_rate=frs[t])
        rec.append(dict(chosen=chosen, fire=fire, mask=mask.clone()))
    if hasattr(model, "message_gain"):
        model.message_gain = gain
    per = loss_premult_rgba(state[:, :4], target.unsqueeze(0).expand_as(state[:, :4]))
    loss = per.mean()
    model.zero_grad(set_to_none=True)
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    return state.detach(), loss.detach(), leaf.grad.detach(), grads, rec


def save_bptt_case(name, model, knobs, x0, target, steps, frs, use_graph, gain, seed=5):
    model = model.train()
    out, loss, gx, grads, rec = _bptt(model, x0, target, steps, frs, use_graph, gain, seed)
    m64 = copy.deepcopy(model).double()
    out64, loss64, gx64, grads64, _ = _bptt(m64, x0.double(), target.double(), steps, frs,
                                            use_graph, gain, seed)
    T = len(rec)
    B, C, H, W = x0.shape
    K = len(rec[0]["chosen"])
    fire = np.zeros((T, B, 1, H, W), np.uint8)
    for t, r in enumerate(rec):
        if r["fire"] is not None:
            fire[t, r["mask"].numpy()] = r["fire"].numpy().astype(np.uint8)
    fields = {"w:" + k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    fields.update(x_in=x0.numpy(), target=target.numpy(), x_out=out.numpy(), x_out_f64=out64.numpy(),
                  loss=loss.numpy(), loss_f64=loss64.numpy(), gx=gx.numpy(), gx_f64=gx64.numpy(),
                  steps=steps.numpy().astype(np.int32), fire_rates=np.array(frs, np.float64),
                  use_graph=np.array(use_graph, np.uint8),
                  active=np.stack([r["mask"].numpy() for r in rec]).astype(np.uint8),
                  offsets=np.array([r["chosen"] for r in rec], np.int32).reshape(T, K, 2),
                  fire_mask=fire)
    for k, v in grads.items():
        fields["g:" + k] = v.numpy()
        fields["g64:" + k] = grads64[k].numpy()
    meta = dict(knobs, graph=hasattr(model, "graph"), message_gain=gain, name=name, rollout=T,
                seed=seed, grad_keys=sorted(grads))
    fields["meta"] = np.array(json.dumps(meta))
    path = os.path.join(OUT, "bptt_" + name + ".npz")
    np.savez_compressed(path, **fields)
    print(f"bptt_{name}: {os.path.getsize(path)/1024:.0f} KB T={T} loss={float(loss):.6f}")


def main():
    gen = torch.Generator().manual_seed(777)
    latest = load_state(f"{CK_GRAPH}/nca_latest.pt")
    ep380 = load_state(f"{CK_GRAPH}/nca_epoch380.pt")
    classic = load_state(f"{CK_CLASSIC}/nca_epoch980.pt")

    k = dict(BASE)
    m = make_graph(k, latest)
    grown = grow(m, 16, 40, 30, gen)
    x2 = torch.cat([grown, grow(m, 16, 40, 45, gen)], 0)
    save_grad_case("graph_torus_latest_grown_b2_40", m, k, x2, 0.5)
    kz = dict(BASE, zero_padded_shift=True)
    save_grad_case("graph_zeropad_latest_grown_b2_40", make_graph(kz, latest), kz, x2, 0.5)
    k380 = dict(BASE, update_gain=0.08, alpha_thr=0.25, message_gain=0.3, zero_padded_shift=True)
    save_grad_case("graph_zeropad_ep380_b1_40", make_graph(k380, ep380), k380,
                   blob_state(1, 16, 40, 40, gen), 0.5)
    kc = dict(BASE)
    save_grad_case("classic_ep980_b2_32", make_classic(kc, classic), kc, blob_state(2, 16, 32, 32, gen),
                   0.5, graph=False)
    for zp in (False, True):
        for ho in (False, True):
            for a2a in (False, True):
                for gn in (False, True):
                    kk = dict(BASE, zero_padded_shift=zp, hidden_only=ho, alive_to_alive=a2a,
                              use_groupnorm=gn, scaling=0.3)
                    name = f"graph_flags_zp{int(zp)}_ho{int(ho)}_a{int(a2a)}_gn{int(gn)}_b2_20x24"
                    save_grad_case(name, make_graph(kk, None, seed=11), kk, blob_state(2, 16, 20, 24, gen), 0.5)
    k32z = dict(BASE, C=32, r=5, K=16, scaling=0.2, zero_padded_shift=True)
    save_grad_case("graph_zeropad_c32_r5_k16_b1_32", make_graph(k32z, None, 5), k32z,
                   blob_state(1, 32, 32, 32, gen), 0.5)
    k32 = dict(BASE, C=32, r=5, K=16, scaling=0.2)
    save_grad_case("graph_torus_c32_r5_k16_b1_32", make_graph(k32, None, 5), k32,
                   blob_state(1, 32, 32, 32, gen), 0.5)
    k8 = dict(BASE, C=8, Hd=32, d=8, scaling=0.5)
    save_grad_case("graph_torus_c8_hd32_b2_24", make_graph(k8, None, 8), k8, blob_state(2, 8, 24, 24, gen), 0.5)
    kc4 = dict(BASE, C=4, Hd=64, d=4, hidden_only=False, scaling=0.5, zero_padded_shift=True)
    save_grad_case("graph_zeropad_c4_hd64_b2_16", make_graph(kc4, None, 9), kc4,
                   blob_state(2, 4, 16, 16, gen), 0.5)
    save_grad_case("graph_torus_latest_fr1_b1_32", m, k, blob_state(1, 16, 32, 32, gen), 1.0)
    kt = dict(BASE, scaling=0.5)
    save_grad_case("graph_torus_tiny_b3_5x7", make_graph(kt, None, 4), kt, random_state(3, 16, 5, 7, gen), 0.5)
    ktz = dict(kt, zero_padded_shift=True)
    save_grad_case("graph_zeropad_tiny_b3_5x7", make_graph(ktz, None, 4), ktz,
                   random_state(3, 16, 5, 7, gen), 0.5)
    save_grad_case("graph_torus_ragged_b2_17x29", make_graph(kt, None, 6), kt, blob_state(2, 16, 17, 29, gen), 0.6)
    ke = dict(BASE, r=1, K=8, scaling=0.5)
    save_grad_case("graph_r1_nooffsets_b1_16", make_graph(ke, None, 3), ke, blob_state(1, 16, 16, 16, gen), 0.5)
    kcl = dict(BASE, C=12, Hd=48, use_groupnorm=False)
    save_grad_case("classic_c12_hd48_nogn_b2_20", make_classic(kcl, None, 10), kcl,
                   blob_state(2, 12, 20, 20, gen), 0.5, graph=False)

    # BPTT, the trainer's loop: per-sample step counts, masked sub-batch steps, message schedule
    target = torch.rand(4, 32, 32, generator=gen)
    target[:3] *= target[3:4]
    x0 = torch.cat([grow(m, 16, 32, 20, gen) for _ in range(3)], 0)
    steps = torch.tensor([6, 4, 5])
    frs = [0.5, 0.62, 0.9, 0.55, 0.71, 0.8]
    ug = [True, False, False, True, False, False]
    save_bptt_case("graph_torus_latest_b3_32_t6", make_graph(k, latest), k, x0, target, steps, frs, ug, 0.25)
    save_bptt_case("graph_zeropad_latest_b3_32_t6", make_graph(kz, latest), kz, x0, target, steps, frs, ug, 0.25)
    save_bptt_case("classic_ep980_b3_32_t6", make_classic(kc, classic), kc, x0, target, steps,
                   frs, ug, 0.0)


if __name__ == "__main__":
    main()
