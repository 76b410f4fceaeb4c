"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE modules.

Run in the build container only (it needs /root/reference, which does not exist on the GPU
box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Each fixture is data only: the input state, the model weights (a state_dict flattened into
``w:<key>`` arrays), the knobs, the offsets ``random.sample`` drew, the fire mask
``torch.rand`` drew, the reference's fp32 output (and attention map), the same step run by the
reference in float64, and the next ``random.random()`` after the call (the RNG-consumption
contract).  The reference source itself never leaves the container.

Weights come from the reference's shipped checkpoints, loaded with
``torch.load(..., weights_only=True)``, or from a seeded random init.
"""
from __future__ import annotations

import copy
import json
import os
import random
import sys

import numpy as np
import torch

REF = "/root/reference"
sys.path.insert(0, os.path.join(REF, "src"))
sys.dont_write_bytecode = True

from modules.nca import NeuralCA  # noqa: E402  (reference, src/modules/nca.py)
from modules.ncagraph import NeuralCAGraph  # noqa: E402  (reference, src/modules/ncagraph.py)

OUT = os.path.dirname(os.path.abspath(__file__))
CK_GRAPH = f"{REF}/outputs/graphaug_nca/train_inter_loss/gecko/checkpoints"
CK_CLASSIC = f"{REF}/outputs/classic_nca/train_inter_loss/gecko/checkpoints"


def load_state(path):
    return torch.load(path, map_location="cpu", weights_only=True)["model_state"]


def random_state(B, C, H, W, gen):
    """§8d synthetic state: RGB ~ U(0,1), alpha ~ U(0,1), hidden ~ N(0,1)."""
    x = torch.empty(B, C, H, W)
    x[:, :4] = torch.rand(B, 4, H, W, generator=gen)
    if C > 4:
        x[:, 4:] = torch.randn(B, C - 4, H, W, generator=gen)
    return x


def blob_state(B, C, H, W, gen):
    """A partially alive state: random values inside a few discs, dead elsewhere."""
    x = random_state(B, C, H, W, gen)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    alive = torch.zeros(B, 1, H, W)
    for b in range(B):
        for _ in range(3):
            cy = int(torch.randint(0, H, (1,), generator=gen))
            cx = int(torch.randint(0, W, (1,), generator=gen))
            r = max(2, min(H, W) // 5)
            alive[b, 0][((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r] = 1
    x[:, 3:4] *= alive
    return x


def make_graph(knobs, sd=None, seed=0):
    torch.manual_seed(seed)
    m = NeuralCAGraph(
        n_channels=knobs["C"], update_hidden=knobs["Hd"], update_gain=knobs["update_gain"],
        alpha_thr=knobs["alpha_thr"], use_groupnorm=knobs["use_groupnorm"],
        message_gain=knobs["message_gain"], hidden_only=knobs["hidden_only"],
        graph_d_model=knobs["d"], graph_attention_radius=knobs["r"],
        graph_num_neighbors=knobs["K"], graph_alive_to_alive=knobs["alive_to_alive"],
        graph_zero_padded_shift=knobs["zero_padded_shift"])
    if sd is not None:
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not missing and not unexpected, (missing, unexpected)
    else:  # random init with a non-zero last layer (the ctor zero-inits it, ncagraph.py:65)
        with torch.no_grad():
            m.update_net[2].weight.normal_(0, 0.05)
            if knobs["use_groupnorm"]:
                m.norm.weight.uniform_(0.5, 1.5)
                m.norm.bias.normal_(0, 0.2)
            m.graph.query_proj.weight.normal_(0, 0.3)
            m.graph.key_proj.weight.normal_(0, 0.3)
            m.graph.scaling.fill_(knobs.get("scaling", 0.5))
    return m.eval()


def make_classic(knobs, sd=None, seed=0):
    torch.manual_seed(seed)
    m = NeuralCA(n_channels=knobs["C"], update_hidden=knobs["Hd"],
                 update_gain=knobs["update_gain"], alpha_thr=knobs["alpha_thr"],
                 use_groupnorm=knobs["use_groupnorm"])
    if sd is not None:
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not missing and not unexpected, (missing, unexpected)
    else:
        with torch.no_grad():
            m.update_net[2].weight.normal_(0, 0.05)
            if knobs["use_groupnorm"]:
                m.norm.weight.uniform_(0.5, 1.5)
                m.norm.bias.normal_(0, 0.2)
    return m.eval()


def run_step(model, x, fire_rate, graph, return_attention, rng_seed, torch_seed):
    """Run ONE reference step, recording what its RNG calls drew."""
    B, C, H, W = x.shape
    random.seed(rng_seed)
    torch.manual_seed(torch_seed)
    py_state = random.getstate()
    th_state = torch.get_rng_state()
    chosen = []
    if graph:
        k = min(model.graph.num_neighbors, len(model.graph.offsets))
        chosen = random.sample(model.graph.offsets, k) if k > 0 else []
    fire = None
    if fire_rate < 1.0:
        fire = (torch.rand(B, 1, H, W) <= fire_rate)
    random.setstate(py_state)
    torch.set_rng_state(th_state)
    with torch.no_grad():
        if graph:
            res = model(x, fire_rate=fire_rate, return_attention=return_attention)
        else:
            res = model(x, fire_rate=fire_rate)
    rng_next = random.random()
    out, attn = (res if return_attention else (res, None))
    # the same step in float64, same draws
    m64 = copy.deepcopy(model).double()
    random.setstate(py_state)
    torch.set_rng_state(th_state)
    with torch.no_grad():
        if graph:
            r64 = m64(x.double(), fire_rate=fire_rate, return_attention=return_attention)
        else:
            r64 = m64(x.double(), fire_rate=fire_rate)
    out64, attn64 = (r64 if return_attention else (r64, None))
    return chosen, fire, out, attn, out64, attn64, rng_next


def save_case(name, model, knobs, x, fire_rate, *, graph=True, return_attention=False,
              rng_seed=1234, torch_seed=4321, rollout=1, f64=True):
    fields = {}
    sd = model.state_dict()
    for k, v in sd.items():
        fields["w:" + k] = v.detach().cpu().numpy()
    fields["x_in"] = x.numpy()
    chosen_all, fire_all = [], []
    cur = x
    for t in range(rollout):
        chosen, fire, out, attn, out64, attn64, rng_next = run_step(
            model, cur, fire_rate, graph, return_attention, rng_seed + t, torch_seed + t)
        chosen_all.append(chosen)
        fire_all.append(fire.numpy().astype(np.uint8) if fire is not None else None)
        if t == 0:
            fields["x_out1"] = out.numpy()
            if f64:
                fields["x_out1_f64"] = out64.numpy()
            fields["rng_next"] = np.array(rng_next)
            if attn is not None:
                fields["attn"] = attn.numpy()
                if f64:
                    fields["attn_f64"] = attn64.numpy()
        cur = out
    if rollout > 1:
        fields["x_out"] = cur.numpy()
    K = len(chosen_all[0])
    fields["offsets"] = np.array(chosen_all, dtype=np.int32).reshape(rollout, K, 2)
    if fire_all[0] is not None:
        fields["fire_mask"] = np.stack(fire_all, 0)          # [T,B,1,H,W] uint8
    meta = dict(knobs, graph=graph, fire_rate=fire_rate, return_attention=return_attention,
                rng_seed=rng_seed, torch_seed=torch_seed, rollout=rollout, name=name)
    fields["meta"] = np.array(json.dumps(meta))
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **fields)
    print(f"{name}: {os.path.getsize(path)/1024:.0f} KB  K={K} shape={tuple(x.shape)}")


BASE = dict(C=16, Hd=128, d=16, r=4, K=8, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
            hidden_only=True, alive_to_alive=True, zero_padded_shift=False, use_groupnorm=True)


def grow(model, C, S, steps, gen):
    """Roll the reference from the trainers' seed (train_graph_augmented_nca.py:108-114) to a
    realistic partially-grown state."""
    x = torch.zeros(1, C, S, S)
    x[:, 3, S // 2, S // 2] = 1.0
    x[:, 4:, S // 2, S // 2] = 0.01 * torch.randn(C - 4, generator=gen)
    random.seed(7)
    torch.manual_seed(7)
    with torch.no_grad():
        for _ in range(steps):
            x = model(x, fire_rate=0.5)
    return x


def main():
    gen = torch.Generator().manual_seed(2024)
    latest = load_state(f"{CK_GRAPH}/nca_latest.pt")
    ep380 = load_state(f"{CK_GRAPH}/nca_epoch380.pt")
    crash = load_state(f"{CK_GRAPH}/nca_crash_ep107_step321.pt")
    classic = load_state(f"{CK_CLASSIC}/nca_epoch980.pt")

    # (1) graph, torus, trained weights, grown state, B=1, 72x72, fire 0.5
    k = dict(BASE)
    m = make_graph(k, latest)
    x = grow(m, 16, 72, 60, gen)
    save_case("graph_torus_latest_grown_b1_72", m, k, x, 0.5)
    # (1b) same weights, synthetic random state (bench distribution), B=1
    save_case("graph_torus_latest_rand_b1_72", m, k, random_state(1, 16, 72, 72, gen), 0.5, f64=False)
    # (2) zero-pad mode (pins the dx-ignored quirk), trained weights, grown state
    kz = dict(BASE, zero_padded_shift=True)
    mz = make_graph(kz, latest)
    save_case("graph_zeropad_latest_grown_b1_72", mz, kz, x, 0.5)
    # (2b) epoch380 (alpha_thr 0.25, gain 0.08, msg 0.3) — the attention debugger's weights
    k380 = dict(BASE, update_gain=0.08, alpha_thr=0.25, message_gain=0.3, zero_padded_shift=True)
    m380 = make_graph(k380, ep380)
    save_case("graph_zeropad_ep380_attn_b1_40", m380, k380, blob_state(1, 16, 40, 40, gen), 0.5,
              return_attention=True)
    # (3) classic, trained weights, B=2, 32x32
    kc = dict(BASE)
    mc = make_classic(kc, classic)
    save_case("classic_ep980_b2_32", mc, kc, blob_state(2, 16, 32, 32, gen), 0.5, graph=False)
    save_case("classic_ep980_fr1_b1_32", mc, kc, blob_state(1, 16, 32, 32, gen), 1.0, graph=False)
    # (4) random init, every flag combination, B=2, 20x24 (ragged vs 16-wide tiles)
    for zp in (False, True):
        for ho in (False, True):
            for a2a in (False, True):
                for gn in (False, True):
                    kk = dict(BASE, zero_padded_shift=zp, hidden_only=ho, alive_to_alive=a2a,
                              use_groupnorm=gn, scaling=0.3)
                    mm = make_graph(kk, None, seed=11)
                    name = f"graph_flags_zp{int(zp)}_ho{int(ho)}_a{int(a2a)}_gn{int(gn)}_b2_20x24"
                    save_case(name, mm, kk, blob_state(2, 16, 20, 24, gen), 0.5)
    # (5) C=32, r=5, K=16, random weights, B=1, 48x48 (config-5 shape class)
    k32 = dict(BASE, C=32, r=5, K=16, scaling=0.2)
    m32 = make_graph(k32, None, seed=5)
    save_case("graph_torus_c32_r5_k16_b1_48", m32, k32, blob_state(1, 32, 48, 48, gen), 0.5)
    k32z = dict(k32, zero_padded_shift=True)
    m32z = make_graph(k32z, None, seed=5)
    save_case("graph_zeropad_c32_r5_k16_b1_48", m32z, k32z, blob_state(1, 32, 48, 48, gen), 0.5,
              return_attention=True)
    # (5b) trained r=5 / K=16 checkpoint (crash ep107)
    kcr = dict(BASE, r=5, K=16, update_gain=0.08, alpha_thr=0.2, message_gain=0.4)
    mcr = make_graph(kcr, crash)
    save_case("graph_torus_crash107_r5k16_b1_40", mcr, kcr, blob_state(1, 16, 40, 40, gen), 0.7)
    # (6) 8-step rollout, per-step offsets and masks, trained weights, B=2, 40x40
    save_case("graph_torus_latest_rollout8_b2_40", m, k, grow(m, 16, 40, 30, gen).repeat(2, 1, 1, 1)
              + 0.0, 0.5, rollout=8)
    save_case("graph_zeropad_latest_rollout8_b2_40", mz, kz,
              grow(m, 16, 40, 30, gen).repeat(2, 1, 1, 1) + 0.0, 0.5, rollout=8)
    # (7) fire_rate 1.0 (no torch RNG), (8) return_attention (torus)
    save_case("graph_torus_latest_fr1_b1_40", m, k, blob_state(1, 16, 40, 40, gen), 1.0)
    save_case("graph_torus_latest_attn_b2_40", m, k, blob_state(2, 16, 40, 40, gen), 0.5,
              return_attention=True)
    # edge cases: no offsets (r=1 -> empty list), K > N_off, tiny & ragged canvases, other C/Hd
    ke = dict(BASE, r=1, K=8, scaling=0.5)
    save_case("graph_r1_nooffsets_b1_16", make_graph(ke, None, 3), ke, blob_state(1, 16, 16, 16, gen), 0.5,
              return_attention=True)
    kk0 = dict(BASE, K=0, scaling=0.5)
    save_case("graph_k0_b1_16", make_graph(kk0, None, 3), kk0, blob_state(1, 16, 16, 16, gen), 0.5)
    kbig = dict(BASE, r=2, K=40, scaling=0.5)      # N_off(r=2) = 16 < K
    save_case("graph_kbig_r2_b1_24", make_graph(kbig, None, 3), kbig, blob_state(1, 16, 24, 24, gen), 0.5)
    kt = dict(BASE, scaling=0.5)
    save_case("graph_torus_tiny_b3_5x7", make_graph(kt, None, 4), kt, random_state(3, 16, 5, 7, gen), 0.5)
    ktz = dict(kt, zero_padded_shift=True)
    save_case("graph_zeropad_tiny_b3_5x7", make_graph(ktz, None, 4), ktz, random_state(3, 16, 5, 7, gen), 0.5)
    save_case("graph_torus_ragged_b3_17x29", make_graph(kt, None, 6), kt, blob_state(3, 16, 17, 29, gen), 0.6)
    k8 = dict(BASE, C=8, Hd=32, d=8, scaling=0.5)
    save_case("graph_torus_c8_hd32_b2_24", make_graph(k8, None, 8), k8, blob_state(2, 8, 24, 24, gen), 0.5)
    kc4 = dict(BASE, C=4, Hd=64, d=4, hidden_only=False, scaling=0.5)
    save_case("graph_torus_c4_hd64_b2_16", make_graph(kc4, None, 9), kc4, blob_state(2, 4, 16, 16, gen), 0.5)
    kcl = dict(BASE, C=12, Hd=48, use_groupnorm=False)
    save_case("classic_c12_hd48_nogn_b2_20", make_classic(kcl, None, 10), kcl,
              blob_state(2, 12, 20, 20, gen), 0.5, graph=False)


if __name__ == "__main__":
    main()
