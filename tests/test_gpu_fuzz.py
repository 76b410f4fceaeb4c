"""GPU parity over seeded random configurations of the module (beyond the golden fixtures' grid):
random batch, canvas (ragged, tiny, non-multiple-of-4), channel count, hidden width, graph radius
and offset count, torus / zero-padded shift, GroupNorm on / off, hidden_only, alive_to_alive,
fire rate and message gain.  Each case runs one module step with the reference's draws
(``random.sample`` of the offsets, ``torch.rand`` for the fire mask) and compares it with the f64
oracle (oracle/nca_oracle.py) at the parity tolerance of tests/test_gpu_parity.py and its
backward against the f64 VJP oracle at tests/test_gpu_grad.py's; the graph cases also run a 3-step
rollout through the C ABI, bitwise against 3 single steps.

The seeds are fixed and the kernels and the oracle deterministic, so the set is the same on
every run.
"""
import random

import numpy as np
import pytest
import torch

from oracle import nca_oracle as O

pytestmark = pytest.mark.gpu

ATOL, RTOL = 2e-6, 1e-5
N_CASES = 32


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


def _config(seed):
    g = np.random.default_rng(1000 + seed)
    graph = bool(g.random() < 0.75)
    C = int(g.choice([4, 8, 12, 16, 16, 16, 20, 32]))
    hidden = int(g.choice([32, 64, 128, 128]))
    B = int(g.integers(1, 4))
    H = int(g.integers(5, 81))
    W = int(g.integers(5, 81))
    while B * H * W > 12000:
        H, W = max(5, H * 3 // 4), max(5, W * 3 // 4)
    return dict(graph=graph, C=C, hidden=hidden, B=B, H=H, W=W,
                radius=int(g.integers(1, 6)), K=int(g.choice([0, 4, 8, 8, 16])),
                zp=bool(g.random() < 0.5), gn=bool(g.random() < 0.8),
                hidden_only=bool(g.random() < 0.7), a2a=bool(g.random() < 0.7),
                fire_rate=float(g.choice([1.0, 0.5, 0.75])), msg=float(g.choice([0.0, 0.25, 0.5])),
                d_model=int(g.choice([8, 16])), gain=float(g.choice([0.05, 0.1])),
                thr=float(g.choice([0.1, 0.12])))


def _model(cfg, dev, seed):
    from graph_neural_cellular_automata_amd import NeuralCA, NeuralCAGraph
    torch.manual_seed(seed)
    if cfg["graph"]:
        m = NeuralCAGraph(cfg["C"], cfg["hidden"], update_gain=cfg["gain"], alpha_thr=cfg["thr"],
                          use_groupnorm=cfg["gn"], message_gain=cfg["msg"], hidden_only=cfg["hidden_only"],
                          graph_d_model=cfg["d_model"], graph_attention_radius=cfg["radius"],
                          graph_num_neighbors=cfg["K"], graph_alive_to_alive=cfg["a2a"],
                          graph_zero_padded_shift=cfg["zp"])
    else:
        m = NeuralCA(cfg["C"], cfg["hidden"], update_gain=cfg["gain"], alpha_thr=cfg["thr"],
                     use_groupnorm=cfg["gn"])
    m = m.to(dev).eval()
    with torch.no_grad():
        m.update_net[2].weight.normal_(0, 0.05)
        if cfg["gn"]:
            m.norm.weight.uniform_(0.5, 1.5)
            m.norm.bias.uniform_(-0.2, 0.2)
    return m


def _state(cfg, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.rand(cfg["B"], cfg["C"], cfg["H"], cfg["W"], device=dev, generator=g)
    x[:, 4:] = torch.randn(cfg["B"], cfg["C"] - 4, cfg["H"], cfg["W"], device=dev, generator=g)
    return x


def _oracle_cfg(cfg):
    return dict(update_gain=cfg["gain"], alpha_thr=cfg["thr"], use_groupnorm=cfg["gn"], graph=cfg["graph"],
                message_gain=cfg["msg"], hidden_only=cfg["hidden_only"], zero_padded_shift=cfg["zp"],
                alive_to_alive=cfg["a2a"])


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_config_step_matches_oracle(dev, seed):
    cfg = _config(seed)
    m = _model(cfg, dev, seed)
    x = _state(cfg, dev, seed)
    # the reference's draws: random.sample of the offsets (graph), then torch.rand for the fire mask
    random.seed(seed)
    chosen = m.graph.sample_offsets() if cfg["graph"] else None
    st = torch.cuda.get_rng_state(dev)
    fire = None
    if cfg["fire_rate"] < 1.0:
        fire = (torch.rand(cfg["B"], 1, cfg["H"], cfg["W"], device=dev) <= cfg["fire_rate"]).float()
    torch.cuda.set_rng_state(st, dev)
    random.seed(seed)
    with torch.no_grad():
        out = m(x, fire_rate=cfg["fire_rate"])
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    ref = O.nca_step(x.cpu().numpy().astype(np.float64), p, _oracle_cfg(cfg), chosen=chosen,
                     fire_mask=None if fire is None else fire.cpu().numpy().astype(np.float64))
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=RTOL, atol=ATOL, err_msg=str(cfg))


@pytest.mark.parametrize("seed", [s for s in range(N_CASES) if _config(s)["graph"]])
def test_random_config_rollout_equals_steps(dev, seed):
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    cfg = _config(seed)
    m = _model(cfg, dev, seed)
    x = _state(cfg, dev, seed).contiguous()
    random.seed(seed)
    offs = [m.graph.sample_offsets() for _ in range(3)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight, b1=m.update_net[0].bias,
                   w2=m.update_net[2].weight, **m.graph.weight_tensors())
    if cfg["gn"]:
        tensors.update(gn_weight=m.norm.weight, gn_bias=m.norm.bias)
    w, keep = S.make_weights(tensors)
    flags = m.graph.flags(False) | (L.USE_GROUPNORM if cfg["gn"] else 0) | (L.HIDDEN_ONLY if cfg["hidden_only"] else 0)

    def desc(t):
        return S.make_desc(B=cfg["B"], C=cfg["C"], H=cfg["H"], W=cfg["W"], hidden=cfg["hidden"],
                           d_model=cfg["d_model"], offsets=offs[t], flags=flags, update_gain=cfg["gain"],
                           alpha_thr=cfg["thr"], message_gain=cfg["msg"], fire_rate=cfg["fire_rate"],
                           fire_mode=L.FIRE_HASH if cfg["fire_rate"] < 1.0 else L.FIRE_NONE,
                           rng_seed=seed, rng_step=t)

    r = S.rollout(desc(0), w, x, 3, offs)
    cur = x
    for t in range(3):
        cur, _ = S.step(desc(t), w, cur)
    assert torch.equal(r, cur), str(cfg)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_random_config_backward_matches_oracle(dev, seed):
    """The module's backward (gnca_step_bwd_f32 through autograd) on the same random configurations
    against the f64 VJP oracle (oracle/nca_oracle_vjp.py), per gradient tensor within
    2e-5 * max|ref| + 1e-6 (tests/test_gpu_grad.py).  A parameter the module leaves without a
    gradient (no offsets drawn, the frozen perception, gate_mlp) must have an all-zero reference."""
    from oracle import nca_oracle_vjp as V
    cfg = _config(seed)
    m = _model(cfg, dev, seed)
    if cfg["graph"]:
        with torch.no_grad():   # pooled-logit gradients of a visible size in zero-pad mode
            m.graph.query_proj.weight.normal_(0, 0.3)
            m.graph.key_proj.weight.normal_(0, 0.3)
    x = _state(cfg, dev, seed).requires_grad_(True)
    gy = torch.randn(x.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(77 + seed))
    random.seed(seed)
    chosen = m.graph.sample_offsets() if cfg["graph"] else None
    st = torch.cuda.get_rng_state(dev)
    fire = None
    if cfg["fire_rate"] < 1.0:
        fire = (torch.rand(cfg["B"], 1, cfg["H"], cfg["W"], device=dev) <= cfg["fire_rate"]).double().cpu().numpy()
    torch.cuda.set_rng_state(st, dev)
    random.seed(seed)
    out = m(x, fire_rate=cfg["fire_rate"])
    (out * gy).sum().backward()
    torch.cuda.synchronize()
    p = {k: v.detach().double().cpu().numpy() for k, v in m.state_dict().items()}
    gx, grads = V.nca_step_vjp(x.detach().double().cpu().numpy(), p, _oracle_cfg(cfg),
                               gy.double().cpu().numpy(), chosen=chosen, fire_mask=fire)
    ref = dict(grads, gx=gx)
    got = {n: q.grad for n, q in m.named_parameters() if q.grad is not None}
    got["gx"] = x.grad
    for k, r in ref.items():
        scale = float(np.abs(r).max())
        if k not in got:
            assert scale == 0.0, (k, scale, cfg)
            continue
        g = got[k].detach().cpu().numpy().reshape(r.shape).astype(np.float64)
        err = float(np.abs(g - r).max())
        assert np.isfinite(g).all(), (k, cfg)
        assert err <= 2e-5 * scale + 1e-6, (k, f"err={err:.3e} scale={scale:.3e}", cfg)
    assert set(got) <= set(ref), (sorted(set(got) - set(ref)), cfg)


def _config_split(seed):
    """The 16-channel, hidden-128 shapes the split (bf16x6) K1 variants serve: canvases of whole
    tiles, graph or classic, radius <= 4, torus or zero-padded shift."""
    g = np.random.default_rng(5000 + seed)
    H, W = [(40, 40), (72, 72), (48, 72), (24, 36), (80, 40), (96, 96), (72, 48), (64, 64)][int(g.integers(0, 8))]
    graph = bool(g.random() < 0.75)
    return dict(graph=graph, C=16, hidden=128, B=int(g.choice([1, 2, 5, 12])), H=H, W=W,
                radius=int(g.integers(1, 5)), K=int(g.choice([4, 8, 8])), zp=bool(g.random() < 0.4),
                gn=bool(g.random() < 0.85), hidden_only=bool(g.random() < 0.8), a2a=bool(g.random() < 0.8),
                fire_rate=float(g.choice([1.0, 0.5])), msg=float(g.choice([0.25, 0.5])),
                d_model=16, gain=float(g.choice([0.05, 0.1])), thr=float(g.choice([0.1, 0.12])))


@pytest.mark.parametrize("seed", range(12))
def test_split_k1_shapes_match_oracle(dev, seed):
    """One module step on the split K1's shapes (random batch, canvas, graph radius, modes) against
    the f64 oracle at the parity tolerance."""
    cfg = _config_split(seed)
    m = _model(cfg, dev, seed)
    x = _state(cfg, dev, seed)
    random.seed(seed)
    chosen = m.graph.sample_offsets() if cfg["graph"] else None
    st = torch.cuda.get_rng_state(dev)
    fire = None
    if cfg["fire_rate"] < 1.0:
        fire = (torch.rand(cfg["B"], 1, cfg["H"], cfg["W"], device=dev) <= cfg["fire_rate"]).float()
    torch.cuda.set_rng_state(st, dev)
    random.seed(seed)
    with torch.no_grad():
        out = m(x, fire_rate=cfg["fire_rate"])
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    ref = O.nca_step(x.cpu().numpy().astype(np.float64), p, _oracle_cfg(cfg), chosen=chosen,
                     fire_mask=None if fire is None else fire.cpu().numpy().astype(np.float64))
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=RTOL, atol=ATOL, err_msg=str(cfg))


@pytest.mark.parametrize("seed", [s for s in range(N_CASES) if _config(s)["graph"]])
def test_random_config_attention_matches_oracle(dev, seed):
    """return_attention=True on the random graph configurations: the state and the normalised
    attention map against the f64 oracle (map within 2e-5, tests/test_gpu_parity.py)."""
    cfg = _config(seed)
    m = _model(cfg, dev, seed)
    x = _state(cfg, dev, seed)
    random.seed(seed)
    chosen = m.graph.sample_offsets()
    st = torch.cuda.get_rng_state(dev)
    fire = None
    if cfg["fire_rate"] < 1.0:
        fire = (torch.rand(cfg["B"], 1, cfg["H"], cfg["W"], device=dev) <= cfg["fire_rate"]).float()
    torch.cuda.set_rng_state(st, dev)
    random.seed(seed)
    with torch.no_grad():
        out, attn = m(x, fire_rate=cfg["fire_rate"], return_attention=True)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    ref, ref_attn = O.nca_step(x.cpu().numpy().astype(np.float64), p, _oracle_cfg(cfg), chosen=chosen,
                               fire_mask=None if fire is None else fire.cpu().numpy().astype(np.float64),
                               return_attention=True)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=RTOL, atol=ATOL, err_msg=str(cfg))
    np.testing.assert_allclose(attn.cpu().numpy(), ref_attn, rtol=0, atol=2e-5, err_msg=str(cfg))


@pytest.mark.parametrize("seed", range(0, N_CASES, 2))
def test_random_config_masked_step_equals_subbatch(dev, seed):
    """The active-sample mask (the trainers' x[m] = model(x[m])) on the random configurations: the
    masked module step equals the step of the active sub-batch bitwise, inactive samples pass through
    (uniform fire draws on the whole batch, as the module's mask contract says)."""
    cfg = dict(_config(seed), B=4)
    m = _model(cfg, dev, seed)
    x = _state(cfg, dev, seed)
    active = torch.tensor([True, False, True, True], device=dev)
    random.seed(seed)
    st = torch.cuda.get_rng_state(dev)
    with torch.no_grad():
        out = m(x, fire_rate=1.0, active=active)
    torch.cuda.set_rng_state(st, dev)
    random.seed(seed)
    with torch.no_grad():
        sub = m(x[active].contiguous(), fire_rate=1.0)
    assert torch.equal(out[active], sub), str(cfg)
    assert torch.equal(out[~active], x[~active])


@pytest.mark.parametrize("seed", range(10))
def test_split_k1_rollout_plans_equal_steps(dev, seed):
    """Rollouts of the split K1's shapes at batches that take every rollout plan (the dense fold of
    small batches, the compact field on one stream, the two-stream sub-batch pipeline), 4 steps,
    bitwise against 4 single steps; the plan is recorded in the assertion message."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    cfg = _config_split(seed)
    cfg["B"] = [4, 8, 64, 160, 384][seed % 5]
    cfg["graph"] = seed % 3 != 2
    m = _model(cfg, dev, seed)
    x = _state(cfg, dev, seed).contiguous()
    random.seed(seed)
    offs = [m.graph.sample_offsets() if cfg["graph"] else [] for _ in range(4)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight, b1=m.update_net[0].bias,
                   w2=m.update_net[2].weight)
    if cfg["graph"]:
        tensors.update(m.graph.weight_tensors())
    if cfg["gn"]:
        tensors.update(gn_weight=m.norm.weight, gn_bias=m.norm.bias)
    w, keep = S.make_weights(tensors)
    flags = ((m.graph.flags(False) | (L.HIDDEN_ONLY if cfg["hidden_only"] else 0)) if cfg["graph"] else 0) | \
        (L.USE_GROUPNORM if cfg["gn"] else 0)

    def desc(t):
        return S.make_desc(B=cfg["B"], C=16, H=cfg["H"], W=cfg["W"], hidden=128, d_model=16,
                           offsets=offs[t], flags=flags, update_gain=cfg["gain"], alpha_thr=cfg["thr"],
                           message_gain=cfg["msg"] if cfg["graph"] else 0.0, fire_rate=cfg["fire_rate"],
                           fire_mode=L.FIRE_HASH if cfg["fire_rate"] < 1.0 else L.FIRE_NONE,
                           rng_seed=seed, rng_step=t)

    plan = (S.k1_variant(desc(0))[0], "subs", S.rollout_subs(desc(0)), "fold", S.rollout_fold(desc(0)),
            "compact", S.rollout_compact(desc(0)))
    r = S.rollout(desc(0), w, x, 4, offs)
    cur = x
    for t in range(4):
        cur, _ = S.step(desc(t), w, cur)
    assert torch.equal(r, cur), (plan, cfg)
