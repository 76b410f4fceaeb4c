"""Benchmark: cell-updates/s of the graph-augmented NCA rollout on MI355X (BASELINE.json metric).

Workload (BASELINE.json north_star): graph-augmented NCA, 16 channels, 72x72,
torus offsets, r=4, K=8, update_hidden 128, fire_rate 0.5, pool batch B=1024 per GPU (the
roofline headline configuration).  One benchmark "step" = one CA step over the whole batch.
Per-step host work (the Python ``random.sample`` offset draw, same seed on every rank) is inside
the timed region.  Weights: the reference's trained nca_latest.pt (carried by the committed golden
fixture); state: synthetic (RGB, alpha ~ U(0,1), hidden ~ N(0,1)).  Fire masks come from the
counter RNG keyed by global sample index, so the N-GPU run computes exactly the states the
1-GPU run would for the same samples.  ``--config c2|c3|c5`` runs the other BASELINE.json GPU
configs (classic B=8; graph B=8; 32ch 128^2 r=5 K=16) with the same harness.

Multi-GPU: one process per GPU, B samples per rank (weak scaling; ``--scaling strong``: a fixed global
batch B split B/N per rank, C4's fixed pool), no collective on the data path;
barrier + synchronize around the timed region, max time over ranks.  Launched either by
``torch.distributed.run --nproc-per-node N bench.py --gpus N`` or as plain ``bench.py --gpus N``,
which starts the N ranks itself (torch.distributed.run on 127.0.0.1) before touching the GPU.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import platform
import random
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HD, D_MODEL = 128, 16
PIECE = 8   # rollout steps per host call (the next piece's offsets are drawn while this one runs)
GAIN, THR, MSG_GAIN, FIRE = 0.05, 0.12, 0.25, 0.5
PEAK_F32_MFMA = 157.3e12                               # MI355X_MICROARCH.md, FP32 matrix
PEAK_BF16_MFMA = 2.5e15                                # MI355X_MICROARCH.md, BF16 dense
PEAK_HBM = 8.0e12
GOLDEN = os.path.join(ROOT, "tests", "golden")
# BASELINE.json configs as bench workloads (SURVEY.md §8d "configs restated").  "headline" is the
# roofline headline (north_star: B=1024 x 16ch x 72^2 on 1 GPU; weak scaling over GPUs) and the
# default; c2/c3/c5 are the other GPU configs.  Weights: the reference's trained checkpoints
# (classic nca_epoch980.pt, graph nca_latest.pt) or, for C=32, the seeded random init with
# W2 ~ N(0, 0.02), all carried by committed golden fixtures.
WORKLOADS = {
    "headline": dict(graph=True, C=16, H=72, B=1024, R=4, K=8,
                     fixture="graph_torus_latest_grown_b1_72",
                     name="graph-augmented NCA rollout, torus, r=4, K=8, fire 0.5"),
    "c2": dict(graph=False, C=16, H=72, B=8, R=0, K=0, fixture="classic_ep980_b2_32",
               name="classic NCA rollout (BASELINE config 2), fire 0.5"),
    "c3": dict(graph=True, C=16, H=72, B=8, R=4, K=8, fixture="graph_torus_latest_grown_b1_72",
               name="graph-augmented NCA rollout (BASELINE config 3), torus, r=4, K=8, fire 0.5"),
    # the module's default shift (graph_augmentation.py:42 zero_padded_shift=True; the attention
    # debugger's mode): per-sample softmax offset weights (K0) every step, rows shifted with zero fill
    "zeropad": dict(graph=True, zp=True, C=16, H=72, B=1024, R=4, K=8, fixture="graph_zeropad_latest_grown_b1_72",
                    name="graph-augmented NCA rollout, zero-padded shift (the module default), r=4, K=8, fire 0.5"),
    "c5": dict(graph=True, C=32, H=128, B=128, R=5, K=16, fixture="graph_torus_c32_r5_k16_b1_48",
               name="graph-augmented NCA rollout (BASELINE config 5), 32ch, torus, r=5, K=16, "
                    "fire 0.5, pool 1024 sharded 128/GPU"),
}
# per-launch HBM traffic of K1/K2 measured by rocprofv3 PMC counters in separate passes
# (tools/pmc.sh + tools/pmc_traffic.py); counters cannot be read from inside this process
# the passes of the shipped build (round 4's final tag r04h; a round's tags are not in time order, so
# the name is explicit), else the highest-named file
# round 6: the passes of the final build (tools/_s6z.sh) carry the sha256 of the libgnca.so they ran
# (lib_sha16); the line reports whether that is the library this run loaded ("pmc_build_match")
PMC_TAG = os.environ.get("GNCA_PMC_TAG", "r06z")
PMC_TRAFFIC = os.path.join(ROOT, "profiles", f"{PMC_TAG}_pmc_traffic.json")
if not os.path.exists(PMC_TRAFFIC):
    PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r05z_pmc_traffic.json")
if not os.path.exists(PMC_TRAFFIC):
    PMC_TRAFFIC = max(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_pmc_traffic.json")) or
                      [os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")])


def flop_per_cell(wl):
    """MFMA FLOP per cell-update: 2*(3C*Hd + Hd*C + C*C); classic has no C*C."""
    C = wl["C"]
    return 2 * (3 * C * HD + HD * C + (C * C if wl["graph"] else 0))


def pmc_file(config):
    """The committed PMC passes of ``config``: the headline's PMC_TRAFFIC, the other configs'
    profiles/r05_pmc_traffic_<config>.json (tools/pmc.sh with BENCH_ARGS="--config <config>"), or None."""
    if config == "headline":
        return PMC_TRAFFIC
    for f in (os.path.join(ROOT, "profiles", f"{PMC_TAG}_pmc_traffic_{config}.json"),
              os.path.join(ROOT, "profiles", f"r05_pmc_traffic_{config}.json")):
        if os.path.exists(f):
            return f
    return None


def lib_sha16(path):
    """First 16 hex digits of the sha256 of a built library (the build a measurement ran)."""
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_provenance(config, loaded_lib):
    """Which committed PMC passes the line's traffic / MFMA-busy numbers come from, and whether they
    were collected with the very library this run loaded."""
    f = pmc_file(config)
    if f is None:
        return None
    try:
        src = json.load(open(f)).get("lib_sha16")
    except Exception:
        src = None
    here = lib_sha16(loaded_lib)
    return {"file": os.path.relpath(f, ROOT), "pmc_lib_sha16": src, "this_run_lib_sha16": here,
            "pmc_build_match": bool(src) and src == here}


def pmc_traffic(kernel, config="headline"):
    """HBM bytes per STEP of ``kernel`` from the committed PMC passes: per-launch counter bytes x the
    launches per step the passes ran with (sub-batches; rollout kernels of 2 half-batches)."""
    try:
        d = json.load(open(pmc_file(config)))
        return d["kernels"][kernel]["traffic_bytes"] * d.get("launches_per_step", 1)
    except Exception:
        return None


def pmc_mfma_busy(kernel, cus, config="headline"):
    """MFMA pipe busy fraction of ``kernel`` from the committed PMC pass (profiles/*_pmc_traffic*.json):
    SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over every SIMD: 32 per v_mfma_f32_32x32x16_bf16) /
    (GRBM_GUI_ACTIVE / 8 XCDs = the kernel's cycles, x 4 SIMDs x CUs)."""
    try:
        f = pmc_file(config)
        c = json.load(open(f))["kernels"][kernel]["counters"]
        busy, grbm = c["SQ_VALU_MFMA_BUSY_CYCLES"], c["GRBM_GUI_ACTIVE"]
        return {"value": busy / (grbm / 8 * 4 * cus), "source": os.path.relpath(f, ROOT),
                "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 4 SIMDs x CUs)"}
    except Exception:
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--gpu-warmup-ms", type=float, default=200.0,
                    help="untimed rollout steps on a copy of the start state for this long before the W "
                         "warmup steps: the GPU clocks ramp up over the first ~10-20 ms after idle "
                         "(20 timed steps after 5 warmup steps: 8.47 G/s without, 9.57 G/s with)")
    ap.add_argument("--config", default="headline", choices=sorted(WORKLOADS),
                    help="rollout workload (BASELINE.json configs); default: the roofline headline")
    ap.add_argument("--batch", type=int, default=None,
                    help="samples per GPU (weak scaling) or in the whole job (strong); default: the config's")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak (default): --batch samples per GPU, the job grows with N.  strong: a fixed "
                         "global batch (--batch, default the config's: C4's pool of 1024) split B/N per "
                         "rank, as a fixed sample pool sharded over N GPUs")
    ap.add_argument("--size", type=int, default=None, help="canvas (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=24.0,
                    help="wall budget of the CPU baseline (rank 0, N=1 only), split over its entries")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default=None, choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the default for N>1) on a node; gloo only to rehearse N>1 ranks "
                         "on one GPU.  Given explicitly at N=1, a world-1 process group of that backend "
                         "is initialised too, so the collective code paths (the training gradient "
                         "all-reduce) run through it")
    ap.add_argument("--mode", default="rollout", choices=["rollout", "train", "regen"],
                    help="rollout: the BASELINE.json headline (default).  train: the graph "
                         "trainer's BPTT iteration (SURVEY.md §8f rank 1), steps = iterations.  regen: "
                         "the regeneration diagnostic's return_attention loop (SURVEY.md §8f rank 4; "
                         "B=1, --size canvas, steps = CA steps, one damage at step 120)")
    ap.add_argument("--train-batch", type=int, default=16, help="train: samples per GPU (config.json)")
    ap.add_argument("--train-size", type=int, default=40, help="train: canvas (config.json img_size)")
    args = ap.parse_args()
    args.pg1 = args.dist_backend is not None   # N=1 with an explicit backend: a world-1 process group
    if args.dist_backend is None:
        args.dist_backend = "nccl"
    return args


def load_weights(dev, wl=None):
    wl = wl or WORKLOADS["headline"]
    z = np.load(os.path.join(GOLDEN, wl["fixture"] + ".npz"), allow_pickle=False)
    return {k[2:]: torch.from_numpy(z[k]).to(dev) for k in z.files if k.startswith("w:")}


def weight_struct(w, wl):
    from graph_neural_cellular_automata_amd import step as S
    t = dict(perception=w["perception.conv.weight"], w1=w["update_net.0.weight"],
             b1=w["update_net.0.bias"], w2=w["update_net.2.weight"], gn_weight=w["norm.weight"],
             gn_bias=w["norm.bias"])
    if wl["graph"]:
        t.update(wq=w["graph.query_proj.weight"], bq=w["graph.query_proj.bias"],
                 wk=w["graph.key_proj.weight"], bk=w["graph.key_proj.bias"],
                 wm=w["graph.msg_proj.weight"], bm=w["graph.msg_proj.bias"], scaling=w["graph.scaling"])
    return S.make_weights(t)


def make_desc(wl, B, H, W, offsets, rank, step0=0):
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    flags = L.USE_GROUPNORM | ((L.GRAPH | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE) if wl["graph"] else 0)
    if wl.get("zp"):
        flags |= L.ZERO_PAD_SHIFT
    return S.make_desc(B=B, C=wl["C"], H=H, W=W, hidden=HD, d_model=D_MODEL,
                       offsets=offsets if wl["graph"] else [], flags=flags,
                       update_gain=GAIN, alpha_thr=THR, message_gain=MSG_GAIN, fire_rate=FIRE,
                       fire_mode=L.FIRE_HASH, rng_seed=42, rng_step=step0, sample_base=rank * B)


def _host_cores():
    """(threads to use for "all cores", description): the CPUs this process may run on (affinity),
    capped by a cgroup CPU quota when one is set (a GPU box's share of a larger host)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(per) + 0.5))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    cpu = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, f"{cpu}; affinity {aff} CPUs" + (f", cgroup quota {quota} CPUs" if quota else "")


# BASELINE.md CPU-baseline plan: configs C1-C4 (BASELINE.json configs[0..3]) on the PyTorch-CPU
# restatement of the reference's op sequence, all cores and 1 thread.  Per entry: (graph, B, canvas,
# steps of the config, B of the 1-thread sample) — C4's 1-thread leg times a B=64 slice of the pool
# (one B=1024 step would take ~30 s on one core; the cost per cell does not depend on B there).
CPU_CONFIGS = {
    "C1": dict(graph=False, B=1, H=72, steps=64, B1=1,
               name="classic NCA, B=1, 72^2, 64-step rollout (BASELINE config 1)"),
    "C2": dict(graph=False, B=8, H=72, steps=96, B1=8, name="classic NCA, B=8, 72^2, 96 steps"),
    "C3": dict(graph=True, B=8, H=72, steps=96, B1=8, name="graph NCA torus r=4 K=8, B=8, 72^2, 96 steps"),
    "C4": dict(graph=True, B=1024, H=72, steps=96, B1=64,
               name="graph NCA torus r=4 K=8, pool B=1024, 72^2 (the per-GPU headline shape)"),
}


def cpu_baseline(budget_s: float):
    """The reference's CPU path restated in PyTorch (oracle/torch_cpu_ref.py, pinned by the golden
    fixtures: reference op sequence, fp32, torch.rand fire mask) timed on this host for BASELINE
    configs C1-C4 on all cores and on 1 thread.  Each entry steps the config's rollout until its
    share of ``budget_s`` is spent (at least one step).  ``value`` is C4 on all cores (the workload
    the GPU line measures)."""
    from oracle.torch_cpu_ref import TorchCpuStep, build_offsets
    threads, host = _host_cores()
    gz = np.load(os.path.join(GOLDEN, WORKLOADS["headline"]["fixture"] + ".npz"), allow_pickle=False)
    cz = np.load(os.path.join(GOLDEN, WORKLOADS["c2"]["fixture"] + ".npz"), allow_pickle=False)
    steppers = {
        True: TorchCpuStep({k[2:]: gz[k] for k in gz.files if k.startswith("w:")}, graph=True,
                           update_gain=GAIN, alpha_thr=THR, message_gain=MSG_GAIN),
        False: TorchCpuStep({k[2:]: cz[k] for k in cz.files if k.startswith("w:")}, graph=False,
                            update_gain=GAIN, alpha_thr=THR),
    }
    offs = build_offsets(4)
    old_threads = torch.get_num_threads()
    entries = {}
    per = budget_s / (2 * len(CPU_CONFIGS))
    try:
        for nthr in (threads, 1):
            torch.set_num_threads(nthr)
            for gr_ in (True, False):   # untimed: thread-pool start, first-call kernel setup
                xw = torch.rand(2, 16, 72, 72)
                steppers[gr_](xw, FIRE, random.Random(0).sample(offs, 8) if gr_ else None)
            for name, c in CPU_CONFIGS.items():
                B = c["B"] if nthr == threads else c["B1"]
                g = torch.Generator().manual_seed(0)
                x = torch.rand(B, 16, c["H"], c["H"], generator=g)
                x[:, 4:] = torch.randn(B, 12, c["H"], c["H"], generator=g)
                rr = random.Random(42)
                st = steppers[c["graph"]]
                n = 0
                t0 = time.perf_counter()
                while n < c["steps"]:
                    x = st(x, FIRE, rr.sample(offs, 8) if c["graph"] else None)
                    n += 1
                    if time.perf_counter() - t0 >= per:
                        break
                el = time.perf_counter() - t0
                entries[f"{name}_{'all' if nthr == threads else '1t'}"] = {
                    "value": B * c["H"] * c["H"] * n / el, "threads": nthr, "batch": B, "steps": n,
                    "seconds": round(el, 3), "workload": c["name"]}
    finally:
        torch.set_num_threads(old_threads)
    head = entries["C4_all"]
    return {"value": head["value"], "unit": "cell-updates/s", "cores": threads, "kind": "port",
            "sample": f"PyTorch-CPU restatement of the reference step (oracle/torch_cpu_ref.py, fixture-"
                      f"pinned; fp32, torch.rand fire mask 0.5, trained nca_latest.pt / nca_epoch980.pt "
                      f"weights); value = C4 (graph B=1024 72^2 r=4 K=8) on {threads} threads, "
                      f"{head['steps']} step(s) in {head['seconds']} s; entries: BASELINE configs C1-C4 "
                      f"on all {threads} threads and on 1 thread (C4 1-thread: a B=64 slice); host: {host}",
            "configs": entries}


# The trainer configs (reference configs/config.json "training"/"damage" blocks): the graph
# trainer's canvas for the headline train bench; BASELINE config 5 (32 ch, 128^2, r=5, K=16) adds
# the damage curriculum and the classic trainer's stability phase (the graph
# trainer's own stability block is dead code, train_graph_augmented_nca.py:342-360).
TRAIN_WORKLOADS = {
    "headline": dict(C=16, H=None, R=4, K=8, fixture="graph_torus_latest_grown_b1_72",
                     damage=False, stability=False),
    "c5": dict(C=32, H=128, R=5, K=16, fixture="graph_torus_c32_r5_k16_b1_48",
               damage=True, stability=True),
}
DAMAGE_CFG = {"start_epoch": 100, "prob": 0.3,
              "kinds": {"square": 0.35, "circle": 0.25, "stripes": 0.10, "alpha_drop": 0.15,
                        "saltpepper": 0.05, "gaussian": 0.10},
              "size_min": 6, "size_max": 18, "stripe_width": 6, "alpha_thr": 0.2,
              "alpha_dropout_p": 0.15, "salt_pepper_p": 0.02, "gaussian_softness": 0.35,
              "hidden_noise_sigma": 0.0}


def main_train(args, dev, world, rank):
    """One data-parallel iteration of the graph trainer (train_graph_augmented_nca.py:289-391), on
    the package's device-side pieces: sample a batch from the device-resident pool (this rank's
    shard of the 1024-slot pool), [config c5: the damage curriculum, damage.py:99-138],
    per-sample rollout lengths (48-80 steps, or 200-400 with probability 0.4, config.json), masked
    steps (``active = nca_steps > t``: no sub-batch gather/scatter, no per-step host sync), fire
    rate ~ U(0.5, 0.9) and the message on every 3rd step, premultiplied-RGBA MSE, [config c5: the
    classic trainer's stability phase, train_intermediate_loss.py:257-267: 24 more steps for the
    samples already within 0.01 of the target, + 0.5 * their MSE], loss.backward() through the
    HIP step, one flat RCCL gradient all-reduce, per-parameter grad normalisation, Adam, pool
    replace.  Weak scaling: ``--train-batch`` samples per GPU."""
    import torch.distributed as dist
    import torch.nn.functional as F
    from graph_neural_cellular_automata_amd import NeuralCAGraph
    from graph_neural_cellular_automata_amd.damage import apply_damage_policy_
    from graph_neural_cellular_automata_amd.dp import allreduce_gradients, normalize_gradients_
    from graph_neural_cellular_automata_amd.pool import SamplePool
    from graph_neural_cellular_automata_amd.loss import loss_premult_rgba
    twl = TRAIN_WORKLOADS.get(args.config)
    if twl is None:
        raise SystemExit(f"--mode train supports --config headline|c5, not {args.config}")
    C, R, K = twl["C"], twl["R"], twl["K"]
    torch.manual_seed(7)
    random.seed(42)                       # identical offset draws / fire rates on every rank
    model = NeuralCAGraph(C, HD, update_gain=GAIN, alpha_thr=THR, message_gain=MSG_GAIN,
                          graph_d_model=D_MODEL, graph_attention_radius=R, graph_num_neighbors=K,
                          graph_zero_padded_shift=False).to(dev)
    model.load_state_dict({k: v for k, v in load_weights(dev, twl).items()}, strict=False)
    opt = torch.optim.Adam(model.parameters(), lr=2e-4, weight_decay=1e-5)
    params = [p for p in model.parameters() if p.requires_grad]
    B, H = args.train_batch, twl["H"] or args.train_size
    short, long_, long_prob = (48, 80), (200, 400), 0.4
    stats = {"long_rollouts": 0, "damage_calls": 0, "stability_samples": 0}

    def seed_fn(batch_size=1):            # train_graph_augmented_nca.py:108-114
        g = torch.zeros(batch_size, C, H, H, device=dev)
        g[:, 3:4, H // 2, H // 2] = 1.0
        g[:, 4:, H // 2, H // 2] = 0.01 * torch.randn_like(g[:, 4:, H // 2, H // 2])
        return g

    pool = SamplePool(1024 * world, seed_fn, device=dev, shard=(rank, world))
    # one target for the whole job (every rank trains the same objective); per-rank rollout
    # lengths come from a per-rank generator (each rank's samples are its own)
    target = torch.rand(4, H, H, device=dev, generator=torch.Generator(device=dev).manual_seed(99))
    target[:3] *= target[3:4]
    gen = torch.Generator(device=dev).manual_seed(100 + rank)
    # the stability phase's fire rates: a private stream, so the shared global `random` stream
    # (offset draws, fire rates, short/long regime) stays in lockstep on every rank
    stab_rng = random.Random(4242 + rank)
    cells = [0]
    ar_bytes = [0]   # bytes of the last flat gradient all-reduce (0: no process group)
    # GNCA_TRAIN_PHASES=1 (measurement only): synchronise at the phase boundaries and report the
    # mean wall time of each phase of an iteration on stderr
    phase_t = {} if os.environ.get("GNCA_TRAIN_PHASES") else None

    def mark(name, t_prev):
        if phase_t is None:
            return t_prev
        torch.cuda.synchronize()
        t_now = time.perf_counter()
        phase_t[name] = phase_t.get(name, 0.0) + t_now - t_prev
        return t_now

    def iteration(warm_alloc=False):
        tp = mark("sync", time.perf_counter()) if phase_t is not None else None
        idx, state = pool.sample(B)
        if twl["damage"]:
            apply_damage_policy_(state, DAMAGE_CFG, epoch=DAMAGE_CFG["start_epoch"])
            stats["damage_calls"] += 1
        lo, hi = long_ if random.random() < long_prob else short
        if warm_alloc:   # untimed warmup: the longest rollout once, so the timed iterations run on a
            lo = hi = long_[1]   # grown caching allocator (a trainer's steady state after its first
                                 # long rollout) instead of paying hipMalloc for new activation blocks
        stats["long_rollouts"] += int(lo == long_[0])
        nsteps = torch.randint(lo, hi + 1, (B,), device=dev, generator=gen)
        T = int(nsteps.max().item())
        for t in range(T):
            fr = random.uniform(0.5, 0.9)
            model.message_gain = MSG_GAIN if t % 3 == 0 else 0.0   # message_every = 3
            state = model(state, fire_rate=fr, active=nsteps > t)
        model.message_gain = MSG_GAIN
        tp = mark("sample+rollout", tp)
        cells[0] += int(nsteps.sum().item()) * H * H
        per_sample = loss_premult_rgba(state[:, :4], target[None])   # fused HIP loss (fwd+bwd)
        loss = per_sample.mean()
        if twl["stability"]:
            close = (per_sample < 0.01).detach()
            n = int(close.sum().item())
            run = n > 0
            if world > 1:   # one decision for the job: every rank runs the phase or none does
                flag = torch.tensor([float(n)], device=dev if args.dist_backend == "nccl" else "cpu")
                dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                run = flag.item() > 0
            if run:
                st = state
                for _ in range(24):
                    st = model(st, fire_rate=stab_rng.uniform(0.5, 1.0), active=close)
                if n > 0:
                    loss = loss + 0.5 * F.mse_loss(st[close, :4], target[None].expand(B, -1, -1, -1)[close])
                stats["stability_samples"] += n
                cells[0] += 24 * n * H * H
        tp = mark("loss+stability", tp)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        tp = mark("backward", tp)
        ar_bytes[0] = allreduce_gradients(params)
        normalize_gradients_(params)
        opt.step()
        pool.replace(idx, state.detach())
        mark("allreduce+adam+pool", tp)
        return loss

    for w_ in range(args.warmup):
        iteration(warm_alloc=w_ == 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    cells[0] = 0
    for k_ in stats:
        stats[k_] = 0
    t0 = time.perf_counter()
    if phase_t is not None:
        phase_t.clear()
    for _ in range(args.steps):
        loss = iteration()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if phase_t is not None:
        print("train phases (ms per iteration): " + ", ".join(
            f"{k} {1e3 * v / args.steps:.2f}" for k, v in phase_t.items()), file=sys.stderr, flush=True)
    tot = torch.tensor([float(cells[0])], dtype=torch.float64,
                       device=dev if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        dist.all_reduce(tot)
    if rank == 0:
        extra = ", damage curriculum (config.json), stability phase (24 steps, loss < 0.01)" \
            if twl["damage"] else ""
        line = {
            "metric": "BPTT training cell-updates/sec (forward+backward through the CA step), "
                      "graph trainer iteration",
            "value": float(tot.item()) / el, "unit": "cell-updates/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic target; trainer seed states; "
                    + ("trained nca_latest.pt weights (golden fixture)" if C == 16 else
                       "seeded random-init weights (golden fixture)"),
            "config": {"workload": f"graph trainer iteration ({args.config}): device pool (1024/GPU), "
                                   f"per-sample rollouts 48-80 steps (200-400 w.p. 0.4) via the masked "
                                   f"step, fire U(0.5,0.9), message every 3rd step, premult-RGBA MSE"
                                   f"{extra}, RCCL flat grad all-reduce, grad/||grad||, Adam, pool "
                                   f"replace",
                       "channels": C, "hidden": HD, "height": H, "width": H, "radius": R,
                       "neighbors": K, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"dp{world}"},
            "iterations_per_s": args.steps / el, "final_loss": float(loss.detach()),
            "iteration_stats": stats,
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "allreduce_bytes": ar_bytes[0],
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main_regen(args, dev):
    """The regeneration diagnostic's hot loop (test_graph_augmented_regeneration.py:183-205) on one
    GPU: per step ``state, attn = model(pre_state, fire_rate=0.5, return_attention=True)`` through
    the module (torus mode, :125-140; the trained nca_latest.pt weights, config.json's r=4, K=8),
    plus the loop's ``model.graph.msg_proj(pre_state)`` and its per-channel-group magnitude maps, and
    ONE damage of the policy's square kind at step 120 (:185-189).  Timed: all --steps + 1 model
    calls (the loop runs t = 0..steps), host offset draws and the module's launches included; the
    PNG/MP4 writes are out of scope.  Reported as cell-updates/s = H*W*(steps+1)/time."""
    from graph_neural_cellular_automata_amd import NeuralCAGraph
    from graph_neural_cellular_automata_amd.damage import apply_damage_policy_
    wl = WORKLOADS["headline"]
    H = args.size or wl["H"]
    torch.manual_seed(0)
    random.seed(42)
    model = NeuralCAGraph(16, HD, img_size=H, update_gain=GAIN, alpha_thr=THR, message_gain=MSG_GAIN,
                          graph_d_model=D_MODEL, graph_attention_radius=wl["R"], graph_num_neighbors=wl["K"],
                          graph_zero_padded_shift=False).to(dev).eval()
    model.load_state_dict({k: v for k, v in load_weights(dev, wl).items()}, strict=False)
    dmg = dict(DAMAGE_CFG, prob=1.0, kinds={"square": 1.0})

    def seed():   # utils/nca_init.py:4-7 (make_seed): channels 3.. set to 1 at the centre
        x = torch.zeros(1, 16, H, H, device=dev)
        x[:, 3:, H // 2, H // 2] = 1.0
        return x

    def loop(steps, damage_step):
        state = seed()
        for t in range(steps + 1):
            if t == damage_step:
                apply_damage_policy_(state, dmg, epoch=999999)
            pre_state = state.clone()
            with torch.no_grad():
                state, attn = model(pre_state, fire_rate=FIRE, return_attention=True)
                M = model.graph.msg_proj(pre_state)
                maps = (M[0, :3].abs().mean(dim=0), M[0, 3:4].abs().mean(dim=0), M[0, 4:].abs().mean(dim=0))
        return state, attn, maps

    for _ in range(max(1, args.warmup)):
        loop(min(args.steps, 40), 20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    state, attn, _ = loop(args.steps, 120)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n = args.steps + 1
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    line = {
        "metric": "cell-updates/sec of the regeneration diagnostic's return_attention loop (B=1)",
        "value": H * H * n / el, "unit": "cell-updates/s", "n_gpus": 1, "steps": n, "warmup": args.warmup,
        "ms_per_step": el / n * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "make_seed state, trained nca_latest.pt weights (golden fixture), one square "
                                "damage at step 120",
        "config": {"workload": "test_graph_augmented_regeneration.py loop: model(pre_state, 0.5, "
                               "return_attention=True) + msg_proj maps, torus r=4 K=8",
                   "channels": 16, "hidden": HD, "height": H, "width": H, "batch_per_gpu": 1},
        "k1": S.k1_variant(S.make_desc(
            B=1, C=16, H=H, W=H, hidden=HD, d_model=D_MODEL, offsets=random.Random(1).sample(model.graph.offsets, wl["K"]),
            flags=L.GRAPH | L.USE_GROUPNORM | L.HIDDEN_ONLY | L.ALIVE_TO_ALIVE | L.ATTENTION, update_gain=GAIN,
            alpha_thr=THR, message_gain=MSG_GAIN, fire_rate=FIRE, fire_mode=L.FIRE_RAND_F32))[0],
        "attn_finite": bool(torch.isfinite(attn).all()), "state_finite": bool(torch.isfinite(state).all()),
    }
    print(json.dumps(line), flush=True)


def launch_ranks(args) -> int:
    """``--gpus N`` without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run on 127.0.0.1 and wait for them.  Runs BEFORE any GPU call in this
    process (the parent never touches the GPU and never execs); returns the launcher's exit code."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: {world} ranks launched but --gpus {args.gpus}")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(1, ndev))
    torch.cuda.set_device(dev)
    if world > 1 or args.pg1:
        import torch.distributed as dist
        if world == 1 and "MASTER_PORT" not in os.environ:   # no launcher: a private rendezvous
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
                so.bind(("127.0.0.1", 0))
                os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]),
                                  RANK="0", WORLD_SIZE="1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus
    if args.mode == "train":
        return main_train(args, dev, world, rank)
    if args.mode == "regen":
        return main_regen(args, dev)
    from graph_neural_cellular_automata_amd import _lib as L
    from graph_neural_cellular_automata_amd import step as S
    lib = L.load()
    from graph_neural_cellular_automata_amd.modules.graph_augmentation import GraphAugmentation
    build_offsets = GraphAugmentation._build_offsets   # row-major (dy, dx) table, graph_aug.py:73-83

    wl = WORKLOADS[args.config]
    C, R, K, graph = wl["C"], wl["R"], wl["K"], wl["graph"]
    B = args.batch or wl["B"]
    if args.scaling == "strong":   # a fixed global batch: this rank's share (global samples rank*B ..)
        if B % world:
            raise SystemExit(f"bench: --scaling strong needs the global batch {B} divisible by {world} ranks")
        B //= world
    H = args.size or wl["H"]
    offsets_table = build_offsets(R) if graph else []
    w, w_keep = weight_struct(load_weights(dev, wl), wl)   # w_keep owns the tensors w points at
    # this rank's samples are global samples [rank*B, (rank+1)*B): their start state and fire masks
    # depend on the global index only, so rank 0 of an N-rank run computes the 1-rank run's states
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.rand(B, C, H, H, device=dev, generator=g)
    x[:, 4:] = torch.randn(B, C - 4, H, H, device=dev, generator=g)
    out = torch.empty_like(x)
    scratch = torch.empty_like(x)
    desc0 = make_desc(wl, B, H, H, offsets_table[:K], rank)
    ws = S.workspace(desc0, dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    rr = random.Random(42)  # same seed on every rank: identical offsets, no communication

    tmp = torch.empty_like(x)
    # the fold (gnca_k1_variant arith bit 8): one K1 launch per step, each also finishing the previous
    # step; pieces then hand the last step over unfinished (PENDING_OUT / PENDING_IN) instead of
    # finishing it with a K2 and restarting with a plain K1
    fold = S.rollout_fold(desc0)
    p_in, p_out = (L.ROLLOUT_PENDING_IN, L.ROLLOUT_PENDING_OUT) if fold else (L.ROLLOUT_ALIVE_IN, L.ROLLOUT_ALIVE_OUT)

    def rollout(n, step0, src, dst, record=None, rng=rr):
        """n steps from src into dst, issued in pieces of PIECE steps (gnca_rollout_ex_f32 with the
        alive masks or the pending last step handed over between pieces: bitwise the one-call
        rollout): the host draws the next piece's offsets (graph_augmentation.py:121, timed) while
        the device runs this one."""
        sizes = []   # 1, 2, 4, ... PIECE steps: only the first (one-step) draw is exposed
        while sum(sizes) < n:
            sizes.append(min(1 if not sizes else min(2 * sizes[-1], PIECE), n - sum(sizes)))
        npieces = len(sizes)
        cur = src
        for p in range(npieces):
            m = sizes[p]
            s0 = sum(sizes[:p])
            flat = []
            if graph:
                for _ in range(m):
                    for dy, dx in rng.sample(offsets_table, K):
                        flat += [dy, dx]
            if record is not None:
                record.extend(flat)
            arr = (ctypes.c_int8 * len(flat))(*flat) if flat else None
            d = make_desc(wl, B, H, H, offsets_table[:K], rank, step0 + s0)
            nxt = dst if (npieces - 1 - p) % 2 == 0 else tmp
            fl = (p_in if p > 0 else 0) | (p_out if p + 1 < npieces else 0)
            rc = lib.gnca_rollout_ex_f32(ctypes.byref(d), ctypes.byref(w), m, arr, cur.data_ptr(),
                                         nxt.data_ptr(), scratch.data_ptr(), ws.data_ptr(), ws.numel(),
                                         fl, sptr)
            L.check(rc, "gnca_rollout_ex_f32")
            cur = nxt

    # buffers of the stamped re-run (below), allocated before the GPU warm-up: an allocation between
    # the warm-up and the timed run (or between the timed and the stamped run) idles the GPU, and the
    # run after it starts at ramping clocks
    cap = 16384
    nsub = S.rollout_subs(make_desc(wl, B, H, H, offsets_table[:K], rank, args.warmup))
    stamps = torch.zeros(args.steps * nsub * 4 * cap, dtype=torch.int64, device=dev)
    dst2 = torch.empty_like(x)
    # warmup: the rollout's first W steps, untimed; the K timed steps continue from their state (and
    # fire counters), as one rollout of W + K steps
    start = x
    # GPU warm-up: untimed steps on a copy of the start state (own offset RNG, so the ranks' shared
    # draws stay in lockstep; far fire counters) until the GPU has run for --gpu-warmup-ms
    gw_steps = 0
    if args.gpu_warmup_ms > 0:
        ga, gb = x.clone(), torch.empty_like(x)
        gr = random.Random(7)
        t_w = time.perf_counter()
        while (time.perf_counter() - t_w) * 1e3 < args.gpu_warmup_ms:
            rollout(8, 10 ** 6 + gw_steps, ga, gb, rng=gr)
            torch.cuda.synchronize()
            gw_steps += 8
            ga, gb = gb, ga
        del ga, gb
    if args.warmup > 0:
        start = torch.empty_like(x)
        rollout(args.warmup, 0, x, start)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    def stamped_rollout():
        """The timed rollout again, right after it (same start state, offsets and fire counters),
        through gnca_rollout_stamped_f32; returns its wall ms per step."""
        arr = (ctypes.c_int8 * len(timed_offsets))(*timed_offsets) if timed_offsets else None
        d = make_desc(wl, B, H, H, offsets_table[:K], rank, args.warmup)
        t_s = time.perf_counter()
        L.check(lib.gnca_rollout_stamped_f32(ctypes.byref(d), ctypes.byref(w), args.steps, arr, start.data_ptr(),
                                             dst2.data_ptr(), scratch.data_ptr(), ws.data_ptr(), ws.numel(),
                                             stamps.data_ptr(), cap, sptr), "gnca_rollout_stamped_f32")
        torch.cuda.synchronize()
        return (time.perf_counter() - t_s) * 1e3 / args.steps

    timed_offsets = []
    t0 = time.perf_counter()
    rollout(args.steps, args.warmup, start, out, record=timed_offsets)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    stamped_ms = stamped_rollout()
    cpu_dev = dev if args.dist_backend == "nccl" else "cpu"
    ranks_seen = 1
    rank_sums = [float(out.double().sum())]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cpu_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        one = torch.ones(1, dtype=torch.float64, device=cpu_dev)
        dist.all_reduce(one)
        ranks_seen = int(one.item())
        sums = [torch.zeros(1, dtype=torch.float64, device=cpu_dev) for _ in range(world)]
        dist.all_gather(sums, torch.tensor(rank_sums, dtype=torch.float64, device=cpu_dev))
        rank_sums = [float(v.item()) for v in sums]
    cells = B * H * H
    value = cells * args.steps * world / el

    # --- per-kernel durations of the timed rollout itself: the same rollout again (same start state,
    #     offsets and fire counters; final state checked bitwise) through gnca_rollout_stamped_f32,
    #     where every K1 / K2 workgroup writes wall-clock stamps (100 MHz s_memrealtime) at its start
    #     and end: a launch's duration is max(end) - min(start), with nothing inserted in the stream
    #     between launches.  The stamped run's own wall time is reported beside the timed one. ---
    if not torch.equal(dst2.view(torch.int32), out.view(torch.int32)) and not os.environ.get("GNCA_AB_TIMING_ONLY"):
        raise SystemExit("bench: the stamped rollout differs from the timed rollout")
    sv = stamps.view(args.steps, nsub, 2, cap, 2).cpu().numpy()
    dur = np.zeros((args.steps, nsub, 2))
    tails = []                          # per K1 launch: (last workgroup end - median end) / span
    ivs = ([], [])                      # every K1 / K2 launch's [start, end] in ticks
    first, last = None, None
    for t in range(args.steps):
        for j in range(nsub):
            for k in range(2):
                used = sv[t, j, k, :, 0] > 0
                if not used.any():
                    if fold and k == 1 and t + 1 < args.steps:
                        continue          # the fold: one K2 per rollout, after its last step
                    raise SystemExit(f"bench: no stamps from step {t} sub-batch {j} kernel {k}")
                t0_, t1_ = int(sv[t, j, k, used, 0].min()), int(sv[t, j, k, used, 1].max())
                dur[t, j, k] = (t1_ - t0_) * 1e-5          # 100 MHz ticks -> ms
                if k == 0 and t1_ > t0_:   # the launch's tail: last workgroup end - median end, of its span
                    tails.append((t1_ - float(np.median(sv[t, j, k, used, 1]))) / (t1_ - t0_))
                ivs[k].append((t0_, t1_))
                first = t0_ if first is None else min(first, t0_)
                last = t1_ if last is None else max(last, t1_)
    # per step: the time any K1 (K2) workgroup of the timed rollout was running, i.e. the union of the
    # launches' intervals over the steps (each sub-batch holds 1/nsub of the cells; a sub-batch's K1
    # starts on the CUs the other sub-batch's K1 frees, so the two launches' spans overlap and their
    # sum would exceed the time; a K2 overlaps the other sub-batch's K1)
    def union_ms(iv):
        tot, cur = 0, None
        for a_, b_ in sorted(iv):
            if cur is None or a_ > cur[1]:
                if cur is not None:
                    tot += cur[1] - cur[0]
                cur = [a_, b_]
            else:
                cur[1] = max(cur[1], b_)
        return (tot + (cur[1] - cur[0] if cur is not None else 0)) * 1e-5
    k1_ms, k2_ms = union_ms(ivs[0]) / args.steps, union_ms(ivs[1]) / args.steps
    fold_info = None
    if fold:
        # per step in steady state: the fold K1 (steps 1..K-1; step 0's K1 is the plain one, the
        # rollout's one K2 follows the last step)
        fold_info = {"k1_plain_ms": float(dur[0, 0, 0]), "k2_final_ms": float(dur[-1, 0, 1]),
                     "k1_fold_launches": args.steps - 1}
        if args.steps > 1:
            k1_ms = float(dur[1:, 0, 0].mean())
    span_ms = (last - first) * 1e-5 / args.steps
    del stamps, dst2
    # --- what K1 executes per launch: replay the timed rollout launch by launch (same start state,
    #     offsets and fire counters; the final state is checked bitwise against the timed one) and
    #     count each launch's live cells (keep = pre-alive AND fire: K1 runs the MLP only for them,
    #     the others have dx = 0 exactly) and, for the split K1, its padded 32-cell groups per tile.
    #     Step 0's K1 reads alive bytes from gnca_k_alive, later K1s the previous K2's, exactly as
    #     gnca_rollout_f32 runs them. ---
    d = make_desc(wl, B, H, H, offsets_table[:K], rank, args.warmup)
    k1_name, arith = S.k1_variant(d)
    compact = S.rollout_compact(d)
    tile = None
    if arith == "bf16x6":
        th, tw, _, _, ku = [int(v) for v in k1_name.split("<")[1].rstrip(">").split(",")]   # <TH,TW,RY,RX,KU>
        tile = (th, tw)
    descs = []
    for t in range(args.steps):
        o = timed_offsets[2 * K * t: 2 * K * (t + 1)]
        descs.append(make_desc(wl, B, H, H, [(o[2 * j], o[2 * j + 1]) for j in range(K)] if graph else [],
                               rank, args.warmup + t))
    bufs = [scratch, torch.empty_like(x)]
    ph = L.PHASE_COMPACT if compact else 0

    def launch(t, src, dst, which):
        f = (L.PHASE_K0 | L.PHASE_K1 | (L.PHASE_ALIVE if t > 0 else 0)) if which == 1 else (L.PHASE_K2 | L.PHASE_ALIVE)
        L.check(lib.gnca_step_phases_f32(ctypes.byref(descs[t]), ctypes.byref(w), src.data_ptr(),
                                         dst.data_ptr(), None, None, ws.data_ptr(), ws.numel(), sptr,
                                         f | ph), f"k{which}")

    live = torch.zeros((), dtype=torch.float64, device=dev)
    groups = torch.zeros((), dtype=torch.int64, device=dev)
    src = start
    for t in range(args.steps):
        kp = ((torch.nn.functional.max_pool2d(src[:, 3:4], 3, 1, 1) > THR) & (S.fire_mask(descs[t], dev) != 0))[:, 0]
        live += kp.sum()
        if tile:
            per_tile = kp.reshape(B, H // tile[0], tile[0], H // tile[1], tile[1]).sum(dim=(2, 4))
            groups += ((per_tile + 31) // 32).sum()
        dst = bufs[t % 2]
        launch(t, src, dst, 1)
        launch(t, src, dst, 2)
        src = dst
    torch.cuda.synchronize()
    if not torch.equal(src.view(torch.int32), out.view(torch.int32)) and not os.environ.get("GNCA_AB_TIMING_ONLY"):
        # (GNCA_AB_TIMING_ONLY: timing-only A/B builds, whose outputs are wrong by construction)
        diff = (src != out)
        raise SystemExit(f"bench: the launch-by-launch replay differs from the timed rollout: "
                         f"{int(diff.sum())} values, max |d| {float((src - out).abs().nan_to_num().max()):.3e}, "
                         f"NaN {int(src.isnan().sum())}/{int(out.isnan().sum())}")
    launches = args.steps
    live_frac = float(live) / (cells * launches)
    fpc = flop_per_cell(wl)
    dense_flops = cells * fpc
    live_flops = float(live) / launches * fpc
    # read x, write x'; read dx: dense NCHW, or on the compact field the alpha channel's dense
    # plane and the other channels' live values only
    k2_bytes = cells * 4 * (2 * C + (1 + (C - 1) * live_frac if compact else C))
    # executed MFMA work per launch: live cells are packed into groups of 32 per tile (split K1,
    # v_mfma_f32_32x32x16_bf16 of 32,768 FLOP each per group: 16 channels 108 + 4 for the message,
    # 32 channels 196 + 12; a tile's last group is padded) or, for the f32 K1, the FLOPs per live cell
    if arith == "bf16x6":
        per_group = (112 if ku else 108) if C == 16 else (208 if ku else 196)
        exec_flops = float(groups) / launches * per_group * 32768
        peak_dtype, peak_eq = PEAK_BF16_MFMA, PEAK_BF16_MFMA / 6
        basis = ("bf16 MFMA dense peak (2.5 PFLOP/s) / 6: K1 runs every fp32 product as 6 exact "
                 "bf16 split products (gnca_k1_split.h)")
    else:
        exec_flops = live_flops
        peak_dtype = peak_eq = PEAK_F32_MFMA
        basis = "fp32 MFMA peak (v_mfma_f32_*_f32)"
    k1_s = k1_ms * 1e-3
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    k1_key = "K1F" if fold else "K1"      # the PMC passes' name for the timed K1 (tools/pmc_traffic.py)
    # the PMC passes of this workload: the config's, or for a non-default batch their own (e.g. C4's
    # 128-sample shard: profiles/<tag>_pmc_traffic_b128.json)
    pmc_key = args.config if B == wl["B"] else (f"b{B}" if args.config == "headline" else f"{args.config}_b{B}")
    pmc_busy = pmc_mfma_busy(k1_key, cus, pmc_key)
    k1_traffic = pmc_traffic(k1_key, pmc_key)
    pmc_src = pmc_file(pmc_key)
    roof = {"bound": "mfma", "kernel": k1_name[:-1] + ",fold>" if fold else k1_name, "arith": arith,
            "achieved": live_flops / k1_s / 1e12,
            "peak": peak_eq / 1e12, "unit": "TFLOP/s",
            "frac": live_flops / k1_s / peak_eq,
            "flop_basis": f"executed fp32-equivalent FLOPs: the launch's live cells (keep = fire AND "
                          f"pre-alive, {live_frac:.3f} of all cells; the others have dx = 0 exactly and "
                          f"K1 skips their MLP) x {fpc:,} FLOP (SURVEY.md 8d) / K1's average duration",
            "peak_basis": basis,
            "dense_equiv_frac": dense_flops / k1_s / peak_eq,
            "dense_flop_per_launch": dense_flops, "live_flop_per_launch": live_flops,
            "live_fraction": live_frac,
            "traffic": k1_traffic,
            "traffic_unit": (f"HBM bytes per step (2*FETCH_SIZE+WRITE_SIZE summed over the step's K1 "
                             f"launches, {os.path.relpath(pmc_src, ROOT)})") if pmc_src else None,
            # north_star's "HBM on the fused Sobel+gather stage": that stage is inside K1, which is
            # bound by its MFMA/VALU work (132+ FLOP per byte against the ridge's ~20), so its HBM
            # rate is reported, not targeted
            "k1_hbm_frac": (k1_traffic / (k1_ms * 1e-3) / PEAK_HBM) if k1_traffic else None,
            "k1_ms": k1_ms,
            "k1_ms_source": "per-workgroup s_memrealtime stamps (first instruction .. after the last "
                            "barrier, max - min over the launch's workgroups) in an identical re-run of "
                            "the timed rollout (gnca_rollout_stamped_f32; final state bitwise equal)",
            "mfma_pipe_frac_est": exec_flops / k1_s / peak_dtype,
            "mfma_pipe_note": "executed MFMA FLOPs in the MFMA's dtype (32-cell groups, padding "
                              "included) / that dtype's dense peak",
            "mfma_busy_pmc": pmc_busy,
            "k1_launches_timed": (launches - 1) if fold else launches * nsub,
            "fold": fold_info}
    k2_launch_ms = fold_info["k2_final_ms"] if fold else k2_ms
    roof_k2 = {"bound": "hbm", "kernel": "gnca_k2_finalize", "update_field": "compact" if compact else "dense",
               "achieved": k2_bytes / (k2_launch_ms * 1e-3) / 1e9,
               "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": k2_bytes / (k2_launch_ms * 1e-3) / PEAK_HBM,
               "k2_ms": k2_launch_ms, "bytes_per_launch": k2_bytes,
               "k2_launches_timed": 1 if fold else launches * nsub,
               "note": ("the fold: K2 runs once per rollout (after its last step); every other step's "
                        "finish is inside the next step's K1") if fold else None,
               "traffic": pmc_traffic("K2", pmc_key)}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(args.cpu_seconds)
        metric = ("cell-updates/sec (B·H·W·steps) for 16ch 72×72 rollout at 1/2/4/8 MI355X" if C == 16
                  else f"cell-updates/sec (B·H·W·steps) for {C}ch {H}×{H} rollout")
        wdesc = ("trained nca_latest.pt" if wl["graph"] and C == 16 else
                 "trained classic nca_epoch980.pt" if not wl["graph"] else
                 "seeded random init (W2 ~ N(0,0.02))")
        ms = el / args.steps * 1e3
        line = {
            "metric": metric,
            "value": value, "unit": "cell-updates/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "gpu_warmup": {"ms": args.gpu_warmup_ms, "steps": gw_steps},
            "ms_per_step": ms,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic state (RGB,alpha~U(0,1), hidden~N(0,1)); {wdesc} weights from the "
                    f"committed golden fixture",
            "config": {"workload": wl["name"], "config": args.config,
                       "channels": C, "hidden": HD, "height": H, "width": H,
                       "batch_per_gpu": B, "global_batch": B * world, "parallelism": f"dp{world}"},
            "ranks_seen": ranks_seen, "backend": (args.dist_backend if (world > 1 or args.pg1) else None),
            "rank_state_checksums": rank_sums,
            "k1_k2_ms_vs_step": (k1_ms + k2_ms) / ms,   # > 1 only where sub-batches overlap K2 with K1
            "device_timeline": {"stamped_rollout_ms_per_step": stamped_ms,
                                "k1_tail_frac": float(np.mean(tails)) if tails else None,
                                "first_k1_start_to_last_k2_end_ms_per_step": span_ms,
                                "sub_batches": nsub,
                                "k1_ms": k1_ms, "k2_ms": k2_ms,
                                "gaps_minus_overlap_ms_per_step": span_ms - k1_ms - k2_ms},
            "roofline": roof, "roofline_k2": roof_k2, "cpu_baseline": cpu,
            "pmc_provenance": pmc_provenance(pmc_key, L.LIB_PATH),
        }
        print(json.dumps(line), flush=True)
    if world > 1 or args.pg1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
