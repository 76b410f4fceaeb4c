"""Functional host layer over the C ABI: build descriptors from module state and launch.

Everything here is plumbing around ``libgnca.so``; the arithmetic is in the HIP kernels.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _dev_f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.device.type != "cuda":
        raise RuntimeError(
            f"graph_neural_cellular_automata_amd: {name} is on {t.device}; the NCA step runs only "
            f"on a ROCm GPU (move the model and the state to 'cuda'). There is no CPU path.")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()


def check_state(x: torch.Tensor, C: int) -> torch.Tensor:
    if x.dim() != 4:
        raise ValueError(f"state must be [B,C,H,W], got {tuple(x.shape)}")
    if x.shape[1] != C:
        raise ValueError(f"state has {x.shape[1]} channels, model expects {C}")
    if C < 4:
        raise ValueError("the alive mask reads channel 3: n_channels must be >= 4")
    return _dev_f32(x, "state")


def make_desc(*, B, C, H, W, hidden, d_model, offsets, flags, update_gain, alpha_thr,
              message_gain, fire_rate, fire_mode, gn_eps=1e-3, rng_seed=0, rng_step=0,
              sample_base=0, graph_alpha_thr=None) -> L.StepDesc:
    d = L.StepDesc()
    d.B, d.C, d.H, d.W = int(B), int(C), int(H), int(W)
    d.hidden, d.d_model = int(hidden), int(d_model)
    if len(offsets) > L.MAX_OFFSETS:
        raise ValueError(f"at most {L.MAX_OFFSETS} offsets per step (got {len(offsets)})")
    d.num_offsets = len(offsets)
    for o, (dy, dx) in enumerate(offsets):
        if not (-127 <= dy <= 127 and -127 <= dx <= 127):
            raise ValueError(f"offset {(dy, dx)} out of int8 range")
        d.offsets[2 * o] = int(dy)
        d.offsets[2 * o + 1] = int(dx)
    d.flags = int(flags)
    d.update_gain = float(update_gain)
    d.alpha_thr = float(alpha_thr)
    d.graph_alpha_thr = float(alpha_thr if graph_alpha_thr is None else graph_alpha_thr)
    d.message_gain = float(message_gain)
    d.gn_eps = float(gn_eps)
    d.fire_rate = float(fire_rate)
    d.fire_mode = int(fire_mode)
    d.rng_seed = int(rng_seed) & 0xFFFFFFFFFFFFFFFF
    d.rng_step = int(rng_step)
    d.sample_base = int(sample_base)
    return d


_WCACHE: dict = {}


def _dev_index(device) -> int:
    device = torch.device(device)
    return device.index if device.index is not None else torch.cuda.current_device()


def make_weights(tensors: dict) -> tuple[L.Weights, list]:
    """tensors: name -> device tensor (reference layouts).  Returns the struct and the list of
    contiguous tensors that must stay alive until the launch is enqueued.

    When every tensor is already a contiguous float32 device tensor the struct holds exactly their
    addresses, so it is cached by (name, device, address, shape): a hit rebuilds nothing (in-place
    updates such as optimiser steps keep the addresses).  Only such tensors are looked up or
    stored: the check runs BEFORE the lookup, so a non-contiguous view or a tensor of another dtype
    that happens to sit at a cached address never returns a cached struct.  For cacheable tensors
    the struct is a pure function of the key, so the cache holds no tensor references (the weights
    of a deleted model are freed; a later tensor at the same address gets the same, correct
    struct).  Building the struct was ~20 us of host time per step at the trainer's size."""
    keep = [t for t in tensors.values() if t is not None]
    cacheable = all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in keep)
    key = None
    if cacheable:
        key = tuple((name, t.device.index, t.data_ptr(), tuple(t.shape))
                    for name, t in tensors.items() if t is not None)
        hit = _WCACHE.get(key)
        if hit is not None:
            return hit, keep
    w = L.Weights()
    conv = []
    for name, t in tensors.items():
        if t is None:
            continue
        t = _dev_f32(t.detach(), name)
        conv.append(t)
        setattr(w, name, t.data_ptr())
    if cacheable:
        if len(_WCACHE) >= 256:
            _WCACHE.clear()
        _WCACHE[key] = w
        return w, keep
    return w, conv


_WS_BYTES: dict = {}


def workspace(desc: L.StepDesc, device) -> torch.Tensor:
    # the size depends on the shape class and the offsets' radius (the tile plan), not on the
    # offsets themselves or the knobs' values
    o = desc.offsets[:2 * desc.num_offsets]
    # (the plan also depends on the device's CU count: keyed by device)
    key = (_dev_index(device), desc.B, desc.C, desc.H, desc.W, desc.hidden, desc.d_model, desc.num_offsets, desc.flags,
           desc.message_gain != 0.0, desc.fire_mode,
           max((abs(v) for v in o[0::2]), default=0), max((abs(v) for v in o[1::2]), default=0))
    n = _WS_BYTES.get(key)
    if n is None:
        n = L.load().gnca_workspace_bytes(ctypes.byref(desc))
        if n and len(_WS_BYTES) < 256:
            _WS_BYTES[key] = n
    if n == 0:
        raise L.GncaError(
            f"unsupported step shape: B={desc.B} C={desc.C} H={desc.H} W={desc.W} "
            f"hidden={desc.hidden} (compiled for C <= 32, hidden <= 256)")
    return torch.empty(n, dtype=torch.uint8, device=device)


def k1_variant(desc: L.StepDesc) -> tuple[str, str]:
    """(kernel name, MFMA arithmetic) of the K1 the plan for ``desc`` launches: arithmetic "f32"
    (fp32 MFMA) or "bf16x6" (bf16 MFMA on exact 3-way splits, 6 products per fp32 product)."""
    buf = ctypes.create_string_buffer(128)
    arith = ctypes.c_int32(0)
    L.check(L.load().gnca_k1_variant(ctypes.byref(desc), buf, 128, ctypes.byref(arith)), "gnca_k1_variant")
    return buf.value.decode(), ("bf16x6" if arith.value & 1 else "f32")


def bb_variant(desc: L.StepDesc) -> str:
    """The backward MLP kernel (BB) the backward plan for ``desc`` launches, as
    "gnca_b_mlp<CP,HB,FULL,TH,TW,RY,RX,K,LEAN>" (gnca_bb_variant, host-only)."""
    buf = ctypes.create_string_buffer(128)
    L.check(L.load().gnca_bb_variant(ctypes.byref(desc), buf, 128), "gnca_bb_variant")
    return buf.value.decode()


def rollout_compact(desc: L.StepDesc) -> bool:
    """True when a rollout of ``desc``'s shape runs on the compact update field (K1 packs the live
    cells' dx per tile, K2 unpacks them: GNCA_PHASE_COMPACT)."""
    buf = ctypes.create_string_buffer(128)
    arith = ctypes.c_int32(0)
    L.check(L.load().gnca_k1_variant(ctypes.byref(desc), buf, 128, ctypes.byref(arith)), "gnca_k1_variant")
    return bool(arith.value & 2)


def rollout_subs(desc: L.StepDesc) -> int:
    """Concurrent sub-batches a rollout of ``desc``'s shape runs as (2: one sub-batch's K2 beside
    the other's K1 on two streams; 1: one stream)."""
    buf = ctypes.create_string_buffer(128)
    arith = ctypes.c_int32(0)
    L.check(L.load().gnca_k1_variant(ctypes.byref(desc), buf, 128, ctypes.byref(arith)), "gnca_k1_variant")
    return 2 if arith.value & 4 else 1


def rollout_fold(desc: L.StepDesc, possible: bool = False) -> bool:
    """True when a rollout of ``desc``'s shape folds each step's finish (GroupNorm, tanh * gain,
    residual, post-update alpha gate) into the next step's K1, so one K1 launch per step plus one
    K2 at the end of the rollout (gnca_k1_variant arith bit 8).  ``possible``: whether it can, on
    request (``rollout(..., fold=True)``; arith bit 16) where it is not the default."""
    buf = ctypes.create_string_buffer(128)
    arith = ctypes.c_int32(0)
    L.check(L.load().gnca_k1_variant(ctypes.byref(desc), buf, 128, ctypes.byref(arith)), "gnca_k1_variant")
    return bool(arith.value & (16 if possible else 8))


def stream_ptr(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _active_u8(active, B, device):
    if active is None:
        return None
    if active.device != device or active.dtype not in (torch.bool, torch.uint8) or active.shape != (B,):
        raise ValueError("active must be a [B] bool/uint8 tensor on the state's device")
    active = active.contiguous()
    # a bool tensor is one byte of 0/1 per element: reinterpret, no conversion launch
    return active.view(torch.uint8) if active.dtype == torch.bool else active


def step(desc, weights, x, fire=None, want_attention=False, ws=None, active=None):
    """One step: returns (x_out, attn_or_None).  ``ws``: an optional caller-owned workspace
    (``workspace(desc)``); after the call it holds what ``step_backward(saved=ws)`` reuses.
    ``active``: optional [B] bool/uint8 device mask; inactive samples pass through unchanged
    (gnca_step_masked_f32)."""
    lib = L.load()
    x_out = torch.empty_like(x)
    attn = torch.empty(desc.B, desc.H, desc.W, dtype=torch.float32, device=x.device) \
        if want_attention else None
    if ws is None:
        ws = workspace(desc, x.device)
    act = _active_u8(active, desc.B, x.device)
    if act is not None:
        if want_attention:
            raise ValueError("return_attention is not supported with an active-sample mask")
        rc = lib.gnca_step_masked_f32(ctypes.byref(desc), ctypes.byref(weights), x.data_ptr(),
                                      x_out.data_ptr(), _ptr(fire), act.data_ptr(), ws.data_ptr(),
                                      ws.numel(), stream_ptr(x.device))
        L.check(rc, "gnca_step_masked_f32")
        return x_out, None
    rc = lib.gnca_step_f32(ctypes.byref(desc), ctypes.byref(weights), x.data_ptr(),
                           x_out.data_ptr(), _ptr(fire), _ptr(attn), ws.data_ptr(), ws.numel(),
                           stream_ptr(x.device))
    L.check(rc, "gnca_step_f32")
    return x_out, attn


def message(desc, weights, x, want_attention=False):
    lib = L.load()
    m = torch.empty_like(x)
    attn = torch.empty(desc.B, desc.H, desc.W, dtype=torch.float32, device=x.device) \
        if want_attention else None
    ws = workspace(desc, x.device)
    rc = lib.gnca_message_f32(ctypes.byref(desc), ctypes.byref(weights), x.data_ptr(),
                              m.data_ptr(), _ptr(attn), ws.data_ptr(), ws.numel(),
                              stream_ptr(x.device))
    L.check(rc, "gnca_message_f32")
    return m, attn


def perceive(weight, x):
    lib = L.load()
    B, C, H, W = x.shape
    w = _dev_f32(weight.detach(), "perception weight")
    y = torch.empty(B, 3 * C, H, W, dtype=torch.float32, device=x.device)
    rc = lib.gnca_perceive_f32(B, C, H, W, w.data_ptr(), x.data_ptr(), y.data_ptr(),
                               stream_ptr(x.device))
    L.check(rc, "gnca_perceive_f32")
    return y


def fire_mask(desc, device) -> torch.Tensor:
    """The [B,1,H,W] uint8 fire mask a GNCA_FIRE_HASH step with ``desc`` draws."""
    m = torch.empty(desc.B, 1, desc.H, desc.W, dtype=torch.uint8, device=device)
    L.check(L.load().gnca_fire_mask_u8(ctypes.byref(desc), m.data_ptr(), stream_ptr(device)),
            "gnca_fire_mask_u8")
    return m


def rollout(desc, weights, x, steps: int, offsets_per_step: list, fold: bool = False):
    """``steps`` no-grad steps (GNCA_FIRE_HASH / NONE) in one C call.  ``fold``: fold each step's
    finish into the next K1 even where that is not the default (GNCA_ROLLOUT_FOLD)."""
    lib = L.load()
    k = desc.num_offsets
    flat = [v for offs in offsets_per_step for o in offs for v in o]
    if (desc.flags & L.GRAPH) and k > 0 and len(flat) != steps * 2 * k:
        raise ValueError("offsets_per_step must hold k pairs for every step")
    arr = (ctypes.c_int8 * max(1, len(flat)))(*flat) if flat else None
    out = torch.empty_like(x)
    scratch = torch.empty_like(x)
    ws = workspace(desc, x.device)
    rc = lib.gnca_rollout_ex_f32(ctypes.byref(desc), ctypes.byref(weights), int(steps), arr,
                                 x.data_ptr(), out.data_ptr(), scratch.data_ptr(), ws.data_ptr(),
                                 ws.numel(), L.ROLLOUT_FOLD if fold else 0, stream_ptr(x.device))
    L.check(rc, "gnca_rollout_ex_f32")
    return out


# parameter name (state_dict suffix) -> gnca_grads field
GRAD_FIELDS = {
    "update_net.0.weight": "w1", "update_net.0.bias": "b1", "update_net.2.weight": "w2",
    "norm.weight": "gn_weight", "norm.bias": "gn_bias",
    "graph.query_proj.weight": "wq", "graph.query_proj.bias": "bq",
    "graph.key_proj.weight": "wk", "graph.key_proj.bias": "bk",
    "graph.msg_proj.weight": "wm", "graph.msg_proj.bias": "bm", "graph.scaling": "scaling",
}


def step_backward(desc, weights, x, gy, fire=None, want: dict | None = None, saved=None, active=None,
                  out: dict | None = None):
    """Vector-Jacobian product of one step (gnca_step_bwd_f32).

    ``want`` maps state_dict names (GRAD_FIELDS keys) to the parameter tensors whose gradients
    are wanted; returns ``(gx, {name: grad})`` with grads shaped like the parameters.
    ``saved``: the workspace of the forward ``step(..., ws=saved)`` call on the same inputs
    (skips recomputing the forward's update field).  ``out``: preallocated float32 gradient
    tensors (e.g. views of one flat buffer) for some of the ``want`` names."""
    lib = L.load()
    gy = _dev_f32(gy, "grad_output")
    gx = torch.empty_like(x)
    g = L.Grads()
    given, out = out or {}, {}
    for name, p in (want or {}).items():
        t = given.get(name)
        if t is None:
            t = torch.empty(p.shape, dtype=torch.float32, device=x.device)
        elif t.shape != p.shape or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"gradient buffer for {name} must be contiguous float32 {tuple(p.shape)}")
        out[name] = t
        setattr(g, GRAD_FIELDS[name], t.data_ptr())
    n = lib.gnca_bwd_workspace_bytes(ctypes.byref(desc))
    if n == 0:
        raise L.GncaError(
            f"unsupported step shape for the backward: B={desc.B} C={desc.C} H={desc.H} "
            f"W={desc.W} hidden={desc.hidden}")
    ws = torch.empty(n, dtype=torch.uint8, device=x.device)
    act = _active_u8(active, desc.B, x.device)
    rc = lib.gnca_step_bwd_f32(ctypes.byref(desc), ctypes.byref(weights), x.data_ptr(), _ptr(fire),
                               _ptr(act), gy.data_ptr(), gx.data_ptr(), ctypes.byref(g), _ptr(saved),
                               ws.data_ptr(), ws.numel(), stream_ptr(x.device))
    L.check(rc, "gnca_step_bwd_f32")
    return gx, out
