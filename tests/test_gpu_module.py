"""GPU tests of the nn.Module surface: the reference's call pattern, RNG contract on device,
property checks at the benchmark's full size (B=1024 x 16 x 72 x 72)."""
import ctypes
import random

import numpy as np
import pytest
import torch

from oracle import nca_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


def _trained_like(dev, zp=False, C=16, seed=0):
    from graph_neural_cellular_automata_amd import NeuralCAGraph
    torch.manual_seed(seed)
    m = NeuralCAGraph(C, 128, update_gain=0.05, alpha_thr=0.12, message_gain=0.25,
                      graph_zero_padded_shift=zp).to(dev).eval()
    with torch.no_grad():
        m.update_net[2].weight.normal_(0, 0.05)
    return m


def _state(B, C, H, W, dev, seed=1):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.rand(B, C, H, W, device=dev, generator=g)
    x[:, 4:] = torch.randn(B, C - 4, H, W, device=dev, generator=g)
    return x


@pytest.mark.parametrize("zp", [False, True])
def test_module_forward_rng_contract_and_values(dev, zp):
    m = _trained_like(dev, zp)
    x = _state(2, 16, 40, 40, dev)
    random.seed(5)
    chosen = random.sample(m.graph.offsets, 8)
    nxt = random.random()
    st = torch.cuda.get_rng_state(dev)
    fire = (torch.rand(2, 1, 40, 40, device=dev) <= 0.6).float()
    torch.cuda.set_rng_state(st, dev)
    random.seed(5)
    with torch.no_grad():
        out = m(x, fire_rate=0.6)
    assert random.random() == nxt                       # one random.sample consumed
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    cfg = dict(update_gain=0.05, alpha_thr=0.12, use_groupnorm=True, graph=True,
               message_gain=0.25, hidden_only=True, zero_padded_shift=zp, alive_to_alive=True)
    ref = O.nca_step(x.cpu().numpy().astype(np.float64), p, cfg, chosen=chosen,
                     fire_mask=fire.cpu().numpy().astype(np.float64))
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=2e-6)
    assert not torch.equal(out, x)


def test_relu_keeps_nan_like_torch(dev):
    """A NaN hidden bias: torch.relu keeps NaN (ncagraph.py's update_net), so every updated cell's dx
    is NaN and GroupNorm spreads it over the sample; a NaN-dropping max(h, 0) would not."""
    m = _trained_like(dev)
    with torch.no_grad():
        m.update_net[0].bias[3] = float("nan")
    x = _state(1, 16, 24, 24, dev)
    st = torch.cuda.get_rng_state(dev)
    fire = (torch.rand(1, 1, 24, 24, device=dev) <= 0.5).float()
    torch.cuda.set_rng_state(st, dev)
    random.seed(3)
    chosen = random.sample(m.graph.offsets, 8)
    random.seed(3)
    with torch.no_grad():
        out = m(x, fire_rate=0.5)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    cfg = dict(update_gain=0.05, alpha_thr=0.12, use_groupnorm=True, graph=True,
               message_gain=0.25, hidden_only=True, zero_padded_shift=False, alive_to_alive=True)
    with np.errstate(invalid="ignore"):
        ref = O.nca_step(x.cpu().numpy().astype(np.float64), p, cfg, chosen=chosen,
                         fire_mask=fire.cpu().numpy().astype(np.float64))
    assert np.isnan(ref).any()
    np.testing.assert_array_equal(np.isnan(out.cpu().numpy()), np.isnan(ref))


@pytest.mark.parametrize("shape", [(0, 16, 40, 40), (2, 16, 0, 40)])
def test_empty_state_raises_like_reference(dev, shape):
    """The reference raises RuntimeError on an empty batch (its perception's reshape) and on an
    empty canvas (conv2d's kernel larger than the padded input); its trainer skips empty masks
    (train_graph_augmented_nca.py:305-307).  The module raises a RuntimeError too, launching
    nothing."""
    m = _trained_like(dev)
    x = torch.zeros(shape, device=dev)
    for kw in ({}, {"return_attention": True}):
        with pytest.raises(RuntimeError):
            with torch.no_grad():
                m(x, fire_rate=0.5, **kw)
    torch.cuda.synchronize()
    # the device is still usable afterwards
    with torch.no_grad():
        assert torch.isfinite(m(_state(1, 16, 24, 24, dev), fire_rate=0.5)).all()


def test_torch_rng_consumed_only_when_fire_rate_below_one(dev):
    m = _trained_like(dev)
    x = _state(1, 16, 24, 24, dev)
    st = torch.cuda.get_rng_state(dev)
    with torch.no_grad():
        m(x, fire_rate=1.0)
    assert torch.equal(torch.cuda.get_rng_state(dev), st)
    with torch.no_grad():
        m(x, fire_rate=0.5)
    assert not torch.equal(torch.cuda.get_rng_state(dev), st)


def test_attention_and_message_gain_zero(dev):
    m = _trained_like(dev)
    x = _state(2, 16, 32, 32, dev)
    random.seed(3)
    with torch.no_grad():
        out, attn = m(x, fire_rate=1.0, return_attention=True)
    assert attn.shape == (2, 32, 32)
    assert float(attn.min()) >= 0.0 and float(attn.max()) <= 1.0 + 1e-6
    # message_gain == 0 (the trainer's "no graph" steps) must equal the classic step
    from graph_neural_cellular_automata_amd import NeuralCA
    m.message_gain = 0.0
    classic = NeuralCA(16, 128, update_gain=0.05, alpha_thr=0.12).to(dev)
    classic.load_state_dict({k: v for k, v in m.state_dict().items() if not k.startswith("graph.")})
    with torch.no_grad():
        a = m(x, fire_rate=1.0)
        b = classic(x, fire_rate=1.0)
    assert torch.equal(a, b)


def test_full_size_determinism_and_shard_invariance(dev):
    """B=1024 x 16 x 72 x 72 (the benchmark workload): repeated runs are bitwise identical
    (no float atomics) and a batch split into shards with the global sample index gives the
    same states as the whole batch."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev)
    B = 1024
    x = _state(B, 16, 72, 72, dev, seed=7)
    random.seed(11)
    offs = [random.sample(m.graph.offsets, 8) for _ in range(3)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight, gn_weight=m.norm.weight,
                   gn_bias=m.norm.bias, **m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)

    def roll(xs, base):
        d = S.make_desc(B=xs.shape[0], C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[0],
                        flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                        update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                        fire_mode=L.FIRE_HASH, rng_seed=42, sample_base=base)
        return S.rollout(d, w, xs.contiguous(), 3, offs)

    a = roll(x, 0)
    b = roll(x, 0)
    assert torch.equal(a, b)
    halves = torch.cat([roll(x[:512], 0), roll(x[512:], 512)])
    assert torch.equal(a, halves)
    # rollout API == repeated single steps
    xs = x[:4].contiguous()
    r = roll(xs, 0)
    cur = xs
    for t in range(3):
        d = S.make_desc(B=4, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[t],
                        flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                        update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                        fire_mode=L.FIRE_HASH, rng_seed=42, rng_step=t)
        cur, _ = S.step(d, w, cur)
    assert torch.equal(r, cur)
    # the hashed fire mask agrees with the oracle's definition: check one step vs the oracle
    fm = O.hash_fire_mask(42, 0, 0, 4, 72, 72, 0.5)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    cfg = dict(update_gain=0.05, alpha_thr=0.12, use_groupnorm=True, graph=True,
               message_gain=0.25, hidden_only=True, zero_padded_shift=False, alive_to_alive=True)
    d = S.make_desc(B=4, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[0],
                    flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                    update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                    fire_mode=L.FIRE_HASH, rng_seed=42, rng_step=0)
    one, _ = S.step(d, w, xs)
    ref = O.nca_step(xs.cpu().numpy().astype(np.float64), p, cfg, chosen=offs[0], fire_mask=fm)
    np.testing.assert_allclose(one.cpu().numpy(), ref, rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("graph", [True, False])
def test_compact_rollout_equals_dense_steps(dev, graph):
    """The rollout's compact update field (K1 packs the live cells' dx per tile with per-row live
    masks, K2 unpacks them; GNCA_PHASE_COMPACT) gives bitwise the states of repeated single steps
    on the dense NCHW field, at a batch that plans the large-batch split K1 (24x36 tiles) and in
    the classic step; and the phase API in compact mode equals the rollout."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, seed=6)
    B, steps = 128, 3
    x = _state(B, 16, 72, 72, dev, seed=21)
    random.seed(13)
    offs = [random.sample(m.graph.offsets, 8) if graph else [] for _ in range(steps)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight, gn_weight=m.norm.weight,
                   gn_bias=m.norm.bias)
    if graph:
        tensors.update(m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)
    flags = L.USE_GROUPNORM | ((L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE) if graph else 0)

    def desc(t):
        return S.make_desc(B=B, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[t], flags=flags,
                           update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                           fire_mode=L.FIRE_HASH, rng_seed=42, rng_step=t)

    name, arith = S.k1_variant(desc(0))
    assert arith == "bf16x6", name
    # B=128: one stream on the compact field (its halves are below the sub-batch threshold), which
    # folds by default since round 6
    assert S.rollout_subs(desc(0)) == 1 and S.rollout_fold(desc(0)) and S.rollout_fold(desc(0), possible=True)
    r = S.rollout(desc(0), w, x.contiguous(), steps, offs)
    # the fold on request (each finish inside the next K1, the compact field double-buffered)
    assert torch.equal(S.rollout(desc(0), w, x.contiguous(), steps, offs, fold=True), r)
    cur = x
    for t in range(steps):
        cur, _ = S.step(desc(t), w, cur)
    assert torch.equal(r, cur)
    # the phase API in rollout mode (K1 and K2 calls with PHASE_COMPACT [| PHASE_ALIVE])
    lib = L.load()
    ws = S.workspace(desc(0), dev)
    src, bufs = x.contiguous(), [torch.empty_like(x), torch.empty_like(x)]
    st = torch.cuda.current_stream().cuda_stream
    for t in range(steps):
        d, dst = desc(t), bufs[t % 2]
        for ph in (L.PHASE_K1 | L.PHASE_COMPACT | (L.PHASE_ALIVE if t > 0 else 0),
                   L.PHASE_K2 | L.PHASE_COMPACT | L.PHASE_ALIVE):
            L.check(lib.gnca_step_phases_f32(ctypes.byref(d), ctypes.byref(w), src.data_ptr(),
                                             dst.data_ptr(), None, None, ws.data_ptr(), ws.numel(),
                                             st, ph), "phases")
        src = dst
    assert torch.equal(src, r)


@pytest.mark.parametrize("case", ["all_dead", "all_live", "ragged_batch"])
def test_compact_rollout_edge_cases(dev, case):
    """The compact update field at its extremes: every cell dead (alpha 0: nothing packed, K2
    reads only zeros), every cell live (alpha 1, fire 1.0: every tile row full), and a batch that
    is not a multiple of 8 (no zig-zag K2 order); rollout == repeated dense single steps bitwise."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, seed=8)
    B = 125 if case == "ragged_batch" else 96
    x = _state(B, 16, 72, 72, dev, seed=23)
    if case == "all_dead":
        x[:, 3] = 0.0
    elif case == "all_live":
        x[:, 3] = 1.0
    random.seed(17)
    offs = [random.sample(m.graph.offsets, 8) for _ in range(2)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight, gn_weight=m.norm.weight,
                   gn_bias=m.norm.bias, **m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)
    fr = 1.0 if case == "all_live" else 0.5

    def desc(t):
        return S.make_desc(B=B, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[t],
                           flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                           update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=fr,
                           fire_mode=L.FIRE_HASH if fr < 1.0 else L.FIRE_NONE, rng_seed=5, rng_step=t)

    assert S.rollout_compact(desc(0))
    r = S.rollout(desc(0), w, x.contiguous(), 2, offs)
    cur = x
    for t in range(2):
        cur, _ = S.step(desc(t), w, cur)
    assert torch.equal(r, cur)
    assert torch.isfinite(r).all()


def test_long_rollout_drift(dev):
    """96 steps (the bench's rollout length) against the float64 oracle on the same offsets and
    hashed masks: |hip - oracle| <= 1e-4 and no alive-mask flips."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, seed=3)
    x = _state(2, 16, 32, 32, dev, seed=9)
    random.seed(13)
    T = 96
    offs = [random.sample(m.graph.offsets, 8) for _ in range(T)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight, gn_weight=m.norm.weight,
                   gn_bias=m.norm.bias, **m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)
    d = S.make_desc(B=2, C=16, H=32, W=32, hidden=128, d_model=16, offsets=offs[0],
                    flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                    update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                    fire_mode=L.FIRE_HASH, rng_seed=5)
    got = S.rollout(d, w, x, T, offs).cpu().numpy()
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    cfg = dict(update_gain=0.05, alpha_thr=0.12, use_groupnorm=True, graph=True,
               message_gain=0.25, hidden_only=True, zero_padded_shift=False, alive_to_alive=True)
    ref = x.cpu().numpy().astype(np.float64)
    for t in range(T):
        ref = O.nca_step(ref, p, cfg, chosen=offs[t], fire_mask=O.hash_fire_mask(5, t, 0, 2, 32, 32, 0.5))
    assert np.abs(got - ref).max() <= 1e-4
    np.testing.assert_array_equal(O.alive_mask(got, 0.12), O.alive_mask(ref, 0.12))


def test_fire_mask_u8_matches_oracle_hash(dev):
    """gnca_fire_mask_u8 materialises exactly the oracle's counter-RNG fire mask (with an offset
    sample_base and a later rng_step)."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    d = S.make_desc(B=3, C=16, H=20, W=33, hidden=128, d_model=16, offsets=[], flags=L.GRAPH,
                    update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.37,
                    fire_mode=L.FIRE_HASH, rng_seed=123456789, rng_step=17, sample_base=1000)
    m = S.fire_mask(d, dev).cpu().numpy()
    ref = O.hash_fire_mask(123456789, 17, 1000, 3, 20, 33, 0.37)
    np.testing.assert_array_equal(m.astype(np.float32), ref)


@pytest.mark.parametrize("graph", [True, False])
def test_large_batch_path_vs_oracle(dev, graph):
    """B=256 x 16 x 72 x 72 (the large-batch fixed-geometry K1, 24x36 tiles): three samples of one
    step against the float64 oracle, and a shard split is bitwise equal."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, seed=3)
    B = 256
    x = _state(B, 16, 72, 72, dev, seed=9)
    random.seed(4)
    offs = random.sample(m.graph.offsets, 8) if graph else []
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight, gn_weight=m.norm.weight,
                   gn_bias=m.norm.bias)
    if graph:
        tensors.update(m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)
    flags = L.USE_GROUPNORM | ((L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE) if graph else 0)

    def desc(Bn, base):
        return S.make_desc(B=Bn, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs, flags=flags,
                           update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                           fire_mode=L.FIRE_HASH, rng_seed=42, rng_step=3, sample_base=base)

    out, _ = S.step(desc(B, 0), w, x)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    cfg = dict(update_gain=0.05, alpha_thr=0.12, use_groupnorm=True, graph=graph,
               message_gain=0.25, hidden_only=True, zero_padded_shift=False, alive_to_alive=True)
    fm = O.hash_fire_mask(42, 3, 0, B, 72, 72, 0.5)
    for i in (0, 131, 255):
        ref = O.nca_step(x[i:i + 1].cpu().numpy().astype(np.float64), p, cfg, chosen=offs,
                         fire_mask=fm[i:i + 1])
        np.testing.assert_allclose(out[i:i + 1].cpu().numpy(), ref, rtol=1e-5, atol=2e-6)
    # shard invariance
    lo, _ = S.step(desc(240, 0), w, x[:240].contiguous())
    hi, _ = S.step(desc(16, 240), w, x[240:].contiguous())   # small shard: the small-batch variant
    assert torch.equal(out[:240], lo)
    np.testing.assert_allclose(out[240:].cpu().numpy(), hi.cpu().numpy(), rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("msg", [0.25, 0.0])
def test_c32_split32_path_vs_oracle(dev, msg):
    """BASELINE config 5's shape class (32 ch, 128 x 128, r = 5, K = 16) at B=64 takes the
    32-channel split K1 (gnca_k1_split32, channels staged in two 16-channel phases): two samples
    of one step against the float64 oracle (message on, and message_gain 0 = the no-gather
    variant), and a shard split is bitwise equal."""
    from graph_neural_cellular_automata_amd import NeuralCAGraph
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    torch.manual_seed(5)
    m = NeuralCAGraph(32, 128, update_gain=0.05, alpha_thr=0.12, message_gain=msg,
                      graph_attention_radius=5, graph_num_neighbors=16,
                      graph_zero_padded_shift=False).to(dev).eval()
    with torch.no_grad():
        m.update_net[2].weight.normal_(0, 0.02)
    B, H = 64, 128
    x = _state(B, 32, H, H, dev, seed=13)
    random.seed(8)
    offs = random.sample(m.graph.offsets, 16)
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight, gn_weight=m.norm.weight,
                   gn_bias=m.norm.bias, **m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)

    def desc(Bn, base):
        return S.make_desc(B=Bn, C=32, H=H, W=H, hidden=128, d_model=16, offsets=offs,
                           flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                           update_gain=0.05, alpha_thr=0.12, message_gain=msg, fire_rate=0.5,
                           fire_mode=L.FIRE_HASH, rng_seed=42, rng_step=1, sample_base=base)

    name, arith = S.k1_variant(desc(B, 0))
    assert arith == "bf16x6" and name.startswith("gnca_k1_split32<16,16,"), name
    out, _ = S.step(desc(B, 0), w, x)
    p = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    cfg = dict(update_gain=0.05, alpha_thr=0.12, use_groupnorm=True, graph=True,
               message_gain=msg, hidden_only=True, zero_padded_shift=False, alive_to_alive=True)
    fm = O.hash_fire_mask(42, 1, 0, B, H, H, 0.5)
    for i in (0, 63):
        ref = O.nca_step(x[i:i + 1].cpu().numpy().astype(np.float64), p, cfg, chosen=offs,
                         fire_mask=fm[i:i + 1])
        np.testing.assert_allclose(out[i:i + 1].cpu().numpy(), ref, rtol=1e-5, atol=2e-6)
    lo, _ = S.step(desc(32, 0), w, x[:32].contiguous())
    hi, _ = S.step(desc(32, 32), w, x[32:].contiguous())
    assert torch.equal(out, torch.cat([lo, hi]))
    # the rollout (K2 hands each step's alive masks to the next K1) == repeated single steps
    d0 = desc(B, 0)
    d0.rng_step = 0
    r = S.rollout(d0, w, x, 3, [offs] * 3)
    cur = x
    for t in range(3):
        dt = desc(B, 0)
        dt.rng_step = t
        cur, _ = S.step(dt, w, cur)
    assert torch.equal(r, cur)


def test_masked_step_many_tiles_per_workgroup(dev):
    """The 16-channel split K1 at B=256, 72^2: 1536 tiles of 24x36 over one persistent workgroup per
    CU, so every workgroup walks several tiles and its preparer wave looks ahead past runs of
    inactive samples (next_active).  The masked step's active samples equal the unmasked step's
    bit for bit (samples are independent: per-sample GroupNorm, fire hashed by global sample
    index); inactive samples pass through unchanged."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, seed=3)
    B, H = 256, 72
    x = _state(B, 16, H, H, dev, seed=21)
    random.seed(2)
    offs = random.sample(m.graph.offsets, 8)
    w, keep = S.make_weights(dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                                  b1=m.update_net[0].bias, w2=m.update_net[2].weight,
                                  gn_weight=m.norm.weight, gn_bias=m.norm.bias,
                                  **m.graph.weight_tensors()))
    d = S.make_desc(B=B, C=16, H=H, W=H, hidden=128, d_model=16, offsets=offs,
                    flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                    update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                    fire_mode=L.FIRE_HASH, rng_seed=7, rng_step=3, sample_base=0)
    name = ctypes.create_string_buffer(64)
    assert L.load().gnca_k1_variant(ctypes.byref(d), name, 64, None) == 0
    assert name.value.decode().startswith("gnca_k1_split<24,36")
    g = torch.Generator().manual_seed(4)
    act = torch.rand(B, generator=g) < 0.5
    act[10:40] = False                     # a long run of inactive samples
    act[100:130] = True
    act = act.to(dev)
    full, _ = S.step(d, w, x)
    masked, _ = S.step(d, w, x, active=act)
    assert torch.equal(masked[act], full[act])
    assert torch.equal(masked[~act], x[~act])


@pytest.mark.parametrize("zp", [False, True])
def test_subbatch_rollout_and_pieces_bitwise(dev, zp):
    """A large-batch rollout of a K1 without a fold variant (the 40^2 trainer canvas's 8x20 tiles)
    runs as 2 sub-batches on two streams (one sub-batch's K2 beside the other's K1): bitwise the
    states of repeated single steps; and a rollout issued in pieces with the alive masks handed over
    through the workspace (gnca_rollout_ex_f32 ALIVE_OUT / ALIVE_IN) is bitwise the one-call
    rollout.  Zero-padded shift: the rollout's K2 also hands the next step's K0 the new state's row
    sums (canon_row_sums' order), which single steps compute in K0's own pass: the same bits."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, zp=zp, seed=9)
    B, steps, H = 384, 5, 40
    x = _state(B, 16, H, H, dev, seed=29)
    random.seed(19)
    offs = [random.sample(m.graph.offsets, 8) for _ in range(steps)]
    w, keep = S.make_weights(dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                                  b1=m.update_net[0].bias, w2=m.update_net[2].weight,
                                  gn_weight=m.norm.weight, gn_bias=m.norm.bias,
                                  **m.graph.weight_tensors()))

    def desc(t):
        return S.make_desc(B=B, C=16, H=H, W=H, hidden=128, d_model=16, offsets=offs[t],
                           flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE |
                           (L.ZERO_PAD_SHIFT if zp else 0),
                           update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                           fire_mode=L.FIRE_HASH, rng_seed=3, rng_step=t, sample_base=7)

    assert S.k1_variant(desc(0))[0] == "gnca_k1_split<8,20,4,4,8>"
    assert S.rollout_subs(desc(0)) == 2 and not S.rollout_fold(desc(0))
    r = S.rollout(desc(0), w, x.contiguous(), steps, offs)
    cur = x
    for t in range(steps):
        cur, _ = S.step(desc(t), w, cur)
    assert torch.equal(r, cur)
    # pieces of 2 + 3 steps with the alive hand-over
    lib = L.load()
    ws = S.workspace(desc(0), dev)
    a, b2, scratch = torch.empty_like(x), torch.empty_like(x), torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    for (s0, n, src, dst, fl) in ((0, 2, x, a, L.ROLLOUT_ALIVE_OUT), (2, 3, a, b2, L.ROLLOUT_ALIVE_IN)):
        flat = [v for o in offs[s0:s0 + n] for p in o for v in p]
        arr = (ctypes.c_int8 * len(flat))(*flat)
        L.check(lib.gnca_rollout_ex_f32(ctypes.byref(desc(s0)), ctypes.byref(w), n, arr, src.data_ptr(),
                                        dst.data_ptr(), scratch.data_ptr(), ws.data_ptr(), ws.numel(), fl, st),
                "gnca_rollout_ex_f32")
    assert torch.equal(b2, r)


def test_make_weights_cache_rejects_non_contiguous_at_cached_address(dev):
    """make_weights caches the struct of contiguous fp32 tensors by address; a non-contiguous view
    (or another dtype) at a cached address must not hit the cache: it gets a contiguous copy."""
    from graph_neural_cellular_automata_amd import step as S
    t = torch.randn(16, 16, device=dev)
    w_a, _ = S.make_weights({"w2": t})
    assert w_a.w2 == t.data_ptr()
    v = t.t()                                   # same address, transposed strides
    assert v.data_ptr() == t.data_ptr() and not v.is_contiguous()
    w_b, keep = S.make_weights({"w2": v})
    assert w_b.w2 != t.data_ptr()
    assert any(k.data_ptr() == w_b.w2 and torch.equal(k, v) for k in keep)
    with pytest.raises(TypeError):
        S.make_weights({"w2": t.view(torch.int32)})


@pytest.mark.parametrize("B,graph", [(160, True), (8, True), (8, False), (160, False)])
def test_fold_rollout_pieces_bitwise(dev, B, graph):
    """The fold (each step's finish inside the next step's K1, one launch per step) on the compact
    update field (B=160) and the dense one (B=8, BASELINE configs 2 and 3), graph and classic: a
    rollout issued as a chain of pieces that hand the last step over unfinished (PENDING_OUT /
    PENDING_IN; piece sizes 1, 1, 2, 3 / 4, 3 / 6, 1) is bitwise the one-call rollout and the
    repeated unfused single steps; bad flag combinations are rejected."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    m = _trained_like(dev, seed=12)
    steps = 7
    x = _state(B, 16, 72, 72, dev, seed=31)
    random.seed(23)
    offs = [random.sample(m.graph.offsets, 8) if graph else [] for _ in range(steps)]
    tensors = dict(perception=m.perception.conv.weight, w1=m.update_net[0].weight,
                   b1=m.update_net[0].bias, w2=m.update_net[2].weight,
                   gn_weight=m.norm.weight, gn_bias=m.norm.bias)
    if graph:
        tensors.update(m.graph.weight_tensors())
    w, keep = S.make_weights(tensors)
    flags = L.USE_GROUPNORM | ((L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE) if graph else 0)

    def desc(t):
        return S.make_desc(B=B, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[t], flags=flags,
                           update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                           fire_mode=L.FIRE_HASH, rng_seed=11, rng_step=t, sample_base=3)

    compact = B > 8
    assert S.rollout_compact(desc(0)) == compact
    # small batches fold by default, and so does the compact field where the rollout runs one stream
    # (B=160: its halves are below the sub-batch threshold); otherwise it folds on request
    default_fold = (not compact) or S.rollout_subs(desc(0)) == 1
    assert S.rollout_fold(desc(0)) == default_fold and S.rollout_fold(desc(0), possible=True)
    one = S.rollout(desc(0), w, x.contiguous(), steps, offs, fold=True)
    cur = x
    for t in range(steps):
        cur, _ = S.step(desc(t), w, cur)
    assert torch.equal(one, cur)
    lib = L.load()
    ws = S.workspace(desc(0), dev)
    st = torch.cuda.current_stream().cuda_stream
    scratch = torch.empty_like(x)

    def run(sizes):
        src, s0 = x.contiguous(), 0
        outs = [torch.empty_like(x), torch.empty_like(x)]
        for i, n in enumerate(sizes):
            fl = (L.ROLLOUT_PENDING_IN if i > 0 else 0) | (L.ROLLOUT_PENDING_OUT if i + 1 < len(sizes) else 0) | \
                (L.ROLLOUT_FOLD if compact else 0)
            flat = [v for o in offs[s0:s0 + n] for p in o for v in p]
            arr = (ctypes.c_int8 * len(flat))(*flat) if flat else None
            dst = outs[i % 2]
            L.check(lib.gnca_rollout_ex_f32(ctypes.byref(desc(s0)), ctypes.byref(w), n, arr, src.data_ptr(),
                                            dst.data_ptr(), scratch.data_ptr(), ws.data_ptr(), ws.numel(), fl, st),
                    "gnca_rollout_ex_f32")
            src, s0 = dst, s0 + n
        return src

    assert torch.equal(run([1, 1, 2, 3]), one)
    assert torch.equal(run([4, 3]), one)
    assert torch.equal(run([6, 1]), one)
    # PENDING with ALIVE on the same side, and PENDING on a rollout that does not fold: invalid
    if not (graph and B > 8):
        return
    arr = (ctypes.c_int8 * 16)(*[v for p in offs[0] for v in p])
    for fl in (L.ROLLOUT_PENDING_OUT | L.ROLLOUT_ALIVE_OUT, L.ROLLOUT_PENDING_IN | L.ROLLOUT_ALIVE_IN) + \
            (() if default_fold else (L.ROLLOUT_PENDING_OUT,)):   # (no fold without GNCA_ROLLOUT_FOLD there)
        assert lib.gnca_rollout_ex_f32(ctypes.byref(desc(0)), ctypes.byref(w), 1, arr, x.data_ptr(),
                                       scratch.data_ptr(), torch.empty_like(x).data_ptr(), ws.data_ptr(),
                                       ws.numel(), fl, st) == -1
    # a FOLD request that changes the plan (B=192: two sub-batch streams without it, one fold stream
    # with it) inside an ALIVE chain: every piece of such a chain must run one plan
    d192 = S.make_desc(B=192, C=16, H=72, W=72, hidden=128, d_model=16, offsets=offs[0], flags=flags,
                       update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                       fire_mode=L.FIRE_HASH, rng_seed=11)
    assert S.rollout_subs(d192) > 1 and not S.rollout_fold(d192) and S.rollout_fold(d192, possible=True)
    x192 = _state(192, 16, 72, 72, dev, seed=5)
    ws192 = S.workspace(d192, dev)
    for fl in (L.ROLLOUT_FOLD | L.ROLLOUT_ALIVE_OUT, L.ROLLOUT_FOLD | L.ROLLOUT_ALIVE_IN):
        assert lib.gnca_rollout_ex_f32(ctypes.byref(d192), ctypes.byref(w), 1, arr, x192.data_ptr(),
                                       torch.empty_like(x192).data_ptr(), torch.empty_like(x192).data_ptr(),
                                       ws192.data_ptr(), ws192.numel(), fl, st) == -1
    d8 = S.make_desc(B=8, C=16, H=40, W=40, hidden=128, d_model=16, offsets=offs[0],
                     flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE,
                     update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                     fire_mode=L.FIRE_HASH, rng_seed=11)
    assert not S.rollout_fold(d8, possible=True)   # 40^2: the 8x20 K1 has no fold variant
    x8 = _state(8, 16, 40, 40, dev, seed=2)
    ws8 = S.workspace(d8, dev)
    assert lib.gnca_rollout_ex_f32(ctypes.byref(d8), ctypes.byref(w), 1, arr, x8.data_ptr(),
                                   torch.empty_like(x8).data_ptr(), torch.empty_like(x8).data_ptr(), ws8.data_ptr(),
                                   ws8.numel(), L.ROLLOUT_PENDING_OUT, st) == -1
