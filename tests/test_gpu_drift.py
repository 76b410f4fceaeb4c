"""Long-rollout drift of the SHIPPING kernels against the float64 oracle (a 96-step
rollout within atol 1e-4 and no alive-mask flips).

Each case runs ``gnca_rollout_f32`` at a batch large enough that the planner picks the kernels the
benchmark runs — the bf16x6 split K1 with the compact update field and the K2 -> K1 alive-byte
hand-over — asserts that plan (``S.k1_variant`` / ``S.rollout_compact``), and compares a few samples
with the oracle stepped in float64 on the same offsets and hashed fire masks (global sample index
``sample_base + i``).  Reference path: ``ncagraph.py:106-168`` (graph), ``nca.py:64-105`` (classic).
Weights: the reference's trained checkpoints carried by the golden fixtures (graph nca_latest.pt,
classic nca_epoch980.pt) or, for 32 channels, the fixture's seeded init (W2 ~ N(0, 0.02))."""
import json
import os
import random
import time

import numpy as np
import pytest
import torch

from oracle import nca_oracle as O
from tests.golden_io import Case

pytestmark = pytest.mark.gpu

# case -> (fixture, graph, C, H, B, R, K, steps, samples checked, expected K1, compact field)
CASES = {
    # the headline's shape class: B=96 x 16 x 72^2 graph torus r=4 K=8 -> 576 tiles of 24x36
    "graph_split24x36": ("graph_torus_latest_grown_b1_72", True, 16, 72, 96, 4, 8, 96, (0, 47, 95),
                         "gnca_k1_split<24,36,4,4,8>", True),
    # classic NCA at a large batch (and the trainers' message-off graph steps): the 24x36 classic
    # split K1 (round 6), compact field, sub-batch pipeline
    "classic_split24x36": ("classic_ep980_b2_32", False, 16, 72, 96, 0, 0, 96, (0, 47, 95),
                           "gnca_k1_split<24,36,1,4,0>", True),
    # BASELINE config 2's shape (classic, B=8): the small-tile classic split K1, dense fold
    "classic_split8x24": ("classic_ep980_b2_32", False, 16, 72, 8, 0, 0, 96, (0, 7),
                          "gnca_k1_split<8,24,1,4,0>", False),
    # BASELINE config 3 (graph torus r=4 K=8, B=8, 72^2): the small-batch split K1 on 8x24 tiles,
    # dense update field
    "c3_split8x24": ("graph_torus_latest_grown_b1_72", True, 16, 72, 8, 4, 8, 96, (0, 7),
                     "gnca_k1_split<8,24,4,4,8>", False),
    # the graph trainer's rollout shape (B=16, 40^2, config.json): 8x20 tiles, dense update field
    "trainer_split8x20": ("graph_torus_latest_grown_b1_72", True, 16, 40, 16, 4, 8, 96, (0, 15),
                          "gnca_k1_split<8,20,4,4,8>", False),
    # BASELINE config 5's shape class: 32 ch, 128^2, r=5, K=16 (48 steps: the f64 oracle's time);
    # B=16 gives 1024 tiles, above the compact field's 2-per-CU threshold on 256- and 304-CU parts
    "c5_split32": ("graph_torus_c32_r5_k16_b1_48", True, 32, 128, 16, 5, 16, 48, (0, 15),
                   "gnca_k1_split32<16,16,5,8,16>", True),
    # zero-pad mode (the ctor default, graph_augmentation.py:85-92: rows shifted with zero fill, the
    # column offset ignored; per-sample softmax offset weights from K0): the attention debugger's
    # mode (test_graph_augmented_nca.py:284), on the split K1's zero-padded-shift instance (round 5;
    # the fp32-MFMA runtime K1 before)
    "graph_zeropad_split8x24": ("graph_zeropad_latest_grown_b1_72", True, 16, 72, 8, 4, 8, 96, (0, 7),
                                "gnca_k1_split<8,24,4,4,8>", False, True),
    # the zero-pad LARGE-batch plan (what bench --config zeropad times): the ZP instance
    # of the 24x36 split K1 fed K0's per-sample offset weights, the compact update field, two
    # sub-batch streams, and K2 handing the next step's K0 the new state's row sums (B=192: two
    # sub-batches of 96 samples = 576 tiles each, above the compact field's 2 per CU)
    "graph_zeropad_split24x36": ("graph_zeropad_latest_grown_b1_72", True, 16, 72, 192, 4, 8, 32, (0, 96, 191),
                                 "gnca_k1_split<24,36,4,4,8>", True, True, 2),
}
ARITH = {}   # every case: bf16x6 (the split K1s)
# every case's max |hip - f64| is appended here (JSON lines; the GPU box merges gpurun_out/ back)
DRIFT_LOG = os.environ.get("GNCA_DRIFT_LOG", os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "gpurun_out", "drift_log.jsonl"))
GAIN, THR, MSG, FIRE, SEED = 0.05, 0.12, 0.25, 0.5, 5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("case", sorted(CASES))
def test_shipping_rollout_drift_vs_f64_oracle(dev, case):
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    fx, graph, C, H, B, R, K, T, check, k1_expected, compact, *rest = CASES[case]
    zp = bool(rest and rest[0])
    subs = rest[1] if len(rest) > 1 else None   # the sub-batch streams the rollout must plan
    c = Case(fx)
    p64 = {k: v.astype(np.float64) for k, v in c.weights.items()}
    wt = {k: torch.from_numpy(np.ascontiguousarray(v.astype(np.float32))).to(dev) for k, v in c.weights.items()}
    tensors = dict(perception=wt["perception.conv.weight"], w1=wt["update_net.0.weight"],
                   b1=wt["update_net.0.bias"], w2=wt["update_net.2.weight"],
                   gn_weight=wt["norm.weight"], gn_bias=wt["norm.bias"])
    if graph:
        tensors.update(wq=wt["graph.query_proj.weight"], bq=wt["graph.query_proj.bias"],
                       wk=wt["graph.key_proj.weight"], bk=wt["graph.key_proj.bias"],
                       wm=wt["graph.msg_proj.weight"], bm=wt["graph.msg_proj.bias"],
                       scaling=wt["graph.scaling"])
    w, keep = S.make_weights(tensors)
    # the bench's synthetic state: RGB, alpha ~ U(0,1), hidden ~ N(0,1)
    g = torch.Generator(device=dev).manual_seed(31)
    x = torch.rand(B, C, H, H, device=dev, generator=g)
    x[:, 4:] = torch.randn(B, C - 4, H, H, device=dev, generator=g)
    table = O.build_offsets(R) if graph else []
    rr = random.Random(17)
    offs = [rr.sample(table, K) if graph else [] for _ in range(T)]
    flags = L.USE_GROUPNORM | ((L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE) if graph else 0) | \
        (L.ZERO_PAD_SHIFT if zp else 0)
    base = 1000
    d = S.make_desc(B=B, C=C, H=H, W=H, hidden=128, d_model=16, offsets=offs[0], flags=flags,
                    update_gain=GAIN, alpha_thr=THR, message_gain=MSG, fire_rate=FIRE,
                    fire_mode=L.FIRE_HASH, rng_seed=SEED, rng_step=0, sample_base=base)
    name, arith = S.k1_variant(d)
    assert (name, arith) == (k1_expected, ARITH.get(case, "bf16x6"))
    assert S.rollout_compact(d) == compact, "the rollout's update-field layout"
    if subs is not None:
        assert S.rollout_subs(d) == subs, "the rollout's sub-batch streams"
    got = S.rollout(d, w, x.contiguous(), T, offs).cpu().numpy()
    assert np.isfinite(got).all()
    cfg = dict(update_gain=GAIN, alpha_thr=THR, use_groupnorm=True, graph=graph, message_gain=MSG,
               hidden_only=True, zero_padded_shift=zp, alive_to_alive=True)
    idx = np.array(check)
    ref = x.cpu().numpy()[idx].astype(np.float64)
    for t in range(T):
        fm = np.concatenate([O.hash_fire_mask(SEED, t, base + int(i), 1, H, H, FIRE) for i in idx])
        ref = O.nca_step(ref, p64, cfg, chosen=offs[t] if graph else None, fire_mask=fm)
    err = float(np.abs(got[idx] - ref).max())
    flips = int((O.alive_mask(got[idx], THR) != O.alive_mask(ref, THR)).sum())
    print(f"[drift] {case}: {name}, {T} steps, samples {list(check)}: max |hip - f64| = {err:.3e}")
    os.makedirs(os.path.dirname(DRIFT_LOG), exist_ok=True)
    with open(DRIFT_LOG, "a") as f:
        f.write(json.dumps({"case": case, "k1": name, "compact": compact, "fold": S.rollout_fold(d), "zero_pad": zp,
                            "sub_batches": S.rollout_subs(d),
                            "batch": B, "canvas": H, "steps": T, "samples": list(check),
                            "max_abs_err_vs_f64": err, "mean_abs_err_vs_f64": float(np.abs(got[idx] - ref).mean()),
                            "alive_flips": flips, "tolerance": 1e-4, "time": time.time()}) + "\n")
    assert err <= 1e-4, err
    np.testing.assert_array_equal(O.alive_mask(got[idx], THR), O.alive_mask(ref, THR))


@pytest.mark.parametrize("zp", [False, True])
def test_attention_rollout_drift_vs_f64_oracle(dev, zp):
    """The diagnostics' loops at the headline canvas: one step per call with
    ``return_attention`` (torus: the regeneration diagnostic, test_graph_augmented_regeneration.py:194;
    zero-pad: the attention debugger, test_graph_augmented_nca.py:284-307), 64 steps of B=2 x 72^2 on
    the trained nca_latest.pt weights, the hashed fire mask per step: the state after every step and
    the final step's attention map against the float64 oracle (state atol 1e-4 and no alive flips;
    the min-max normalised map atol 1e-4)."""
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    c = Case("graph_torus_latest_grown_b1_72")
    p64 = {k: v.astype(np.float64) for k, v in c.weights.items()}
    wt = {k: torch.from_numpy(np.ascontiguousarray(v.astype(np.float32))).to(dev) for k, v in c.weights.items()}
    w, keep = S.make_weights(dict(
        perception=wt["perception.conv.weight"], w1=wt["update_net.0.weight"], b1=wt["update_net.0.bias"],
        w2=wt["update_net.2.weight"], gn_weight=wt["norm.weight"], gn_bias=wt["norm.bias"],
        wq=wt["graph.query_proj.weight"], bq=wt["graph.query_proj.bias"], wk=wt["graph.key_proj.weight"],
        bk=wt["graph.key_proj.bias"], wm=wt["graph.msg_proj.weight"], bm=wt["graph.msg_proj.bias"],
        scaling=wt["graph.scaling"]))
    B, H, T = 2, 72, 64
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.rand(B, 16, H, H, device=dev, generator=g)
    x[:, 4:] = torch.randn(B, 12, H, H, device=dev, generator=g)
    table = O.build_offsets(4)
    rr = random.Random(29)
    offs = [rr.sample(table, 8) for _ in range(T)]
    flags = L.USE_GROUPNORM | L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE | L.ATTENTION | \
        (L.ZERO_PAD_SHIFT if zp else 0)
    cfg = dict(update_gain=GAIN, alpha_thr=THR, use_groupnorm=True, graph=True, message_gain=MSG,
               hidden_only=True, zero_padded_shift=zp, alive_to_alive=True)
    ref = x.cpu().numpy().astype(np.float64)
    cur = x
    for t in range(T):
        d = S.make_desc(B=B, C=16, H=H, W=H, hidden=128, d_model=16, offsets=offs[t], flags=flags,
                        update_gain=GAIN, alpha_thr=THR, message_gain=MSG, fire_rate=FIRE,
                        fire_mode=L.FIRE_HASH, rng_seed=SEED, rng_step=t, sample_base=0)
        cur, attn = S.step(d, w, cur, want_attention=True)
        fm = O.hash_fire_mask(SEED, t, 0, B, H, H, FIRE)
        ref, ref_attn = O.nca_step(ref, p64, cfg, chosen=offs[t], fire_mask=fm, return_attention=True)
    got = cur.cpu().numpy()
    err = float(np.abs(got - ref).max())
    aerr = float(np.abs(attn.cpu().numpy() - ref_attn).max())
    flips = int((O.alive_mask(got, THR) != O.alive_mask(ref, THR)).sum())
    name, _ = S.k1_variant(d)
    print(f"[drift] attention {'zero-pad' if zp else 'torus'}: {name}, {T} steps: max |hip - f64| = {err:.3e}, "
          f"attention map {aerr:.3e}, alive flips {flips}")
    os.makedirs(os.path.dirname(DRIFT_LOG), exist_ok=True)
    with open(DRIFT_LOG, "a") as f:
        f.write(json.dumps({"case": "attention_" + ("zeropad" if zp else "torus"), "k1": name, "zero_pad": zp,
                            "batch": B, "canvas": H, "steps": T, "max_abs_err_vs_f64": err,
                            "attention_max_abs_err": aerr, "alive_flips": flips, "tolerance": 1e-4,
                            "time": time.time()}) + "\n")
    assert err <= 1e-4 and aerr <= 1e-4, (err, aerr)
    assert flips == 0
