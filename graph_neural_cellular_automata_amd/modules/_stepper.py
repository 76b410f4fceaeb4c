"""Shared forward of NeuralCA / NeuralCAGraph: descriptor + weights -> one HIP step."""
from __future__ import annotations

import weakref

import torch
import torch.nn as nn

from .. import _lib as L
from .. import step as S


class _ParamPack(torch.autograd.Function):
    """Routes ONE flat gradient to a group of parameters.

    Every step of a rollout hands its parameter gradients to the rollout's shared pack token as
    one flat tensor, so autograd sums them with one add per step and the parameters'
    AccumulateGrad runs once per backward instead of once per parameter per step (12 small
    launches per step at the trainer's size).  The token's value is never read."""

    @staticmethod
    def forward(ctx, sizes, *params):
        ctx.set_materialize_grads(False)
        ctx.sizes = sizes
        ctx.shapes = [p.shape for p in params]
        return params[0].new_empty(sum(sizes))

    @staticmethod
    def backward(ctx, flat):
        if flat is None:
            return (None,) * (1 + len(ctx.shapes))
        return (None, *[g.view(s) for g, s in zip(flat.split(ctx.sizes), ctx.shapes)])


class _Pack:
    """A group of parameters (state_dict names) behind one _ParamPack token."""

    def __init__(self, named):
        self.names = tuple(n for n, _ in named)
        self.params = [p for _, p in named]
        self.sizes = tuple(p.numel() for p in self.params)
        self.token = _ParamPack.apply(self.sizes, *self.params)

    def views(self, flat):
        return {n: g.view(p.shape) for n, g, p in zip(self.names, flat.split(self.sizes), self.params)}


_PACKS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
# fast path: the step's weight-tensor tuple and requires_grad flags -> packs; a hit skips rebuilding
# the named list (7.5 -> 5 us per step).  A weak-keyed side table, not a module attribute: the
# packs hold non-leaf tensors, which would break copy.deepcopy(model)
_PACKS_FAST: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


_SHORT_TO_NAME = {v: k for k, v in S.GRAD_FIELDS.items()}


def param_packs(model: nn.Module, tensors: dict | None = None):
    """(core, graph) packs of the model's trainable parameters that the step backward produces
    (GRAD_FIELDS; ``gate_mlp`` and the frozen perception are never in a pack, so they keep
    ``grad=None`` as in the reference).  ``tensors``: the step's weight tensors by short name
    (``run_step`` has them already; walking ``named_parameters`` costs ~30 us per step).  Cached
    per module: the token only routes gradients, so it stays valid across optimiser steps as
    long as the parameter objects are the same."""
    if tensors is not None:   # fast path: the same parameter objects and requires_grad flags
        vals = tuple(tensors.values())
        flags = tuple(t.requires_grad for t in vals)
        fast = _PACKS_FAST.get(model)
        if fast is not None and fast[0] == flags and len(fast[1]) == len(vals) and \
                all(a is b for a, b in zip(fast[1], vals)):
            return fast[2]
    if tensors is None:
        named = [(n, p) for n, p in model.named_parameters() if n in S.GRAD_FIELDS]
    else:
        named = [(_SHORT_TO_NAME[k], t) for k, t in tensors.items() if k in _SHORT_TO_NAME]
    named = [(n, p) for n, p in named if p.requires_grad]
    dev = named[0][1].device if named else None
    hit = _PACKS.get(model)
    if hit is not None and len(hit[0]) == len(named) and all(a is b for a, (_, b) in zip(hit[0], named)) \
            and hit[2] == dev:
        if tensors is not None:
            _PACKS_FAST[model] = (flags, vals, hit[1])
        return hit[1]
    core = [(n, p) for n, p in named if not n.startswith("graph.")]
    graph = [(n, p) for n, p in named if n.startswith("graph.")]
    packs = (_Pack(core) if core else None, _Pack(graph) if graph else None)
    _PACKS[model] = (tuple(p for _, p in named), packs, dev)
    if tensors is not None:
        _PACKS_FAST[model] = (flags, vals, packs)
    return packs


class _StepFn(torch.autograd.Function):
    """The HIP step as an autograd node (BPTT through the trainers' rollouts).

    Forward: ``gnca_step_f32`` into a workspace that the node keeps (the step's update field and
    GroupNorm partials, ~one state of memory).  Backward: ``gnca_step_bwd_f32`` on that saved
    workspace; everything else (perception, hidden layer, message) is recomputed from the input
    state, so a rollout keeps two state-sized tensors per step alive, far less than the
    reference's per-op activations.  Gradients follow the
    reference's graph of tensors: masks are constants, the perception weight is frozen,
    ``gate_mlp`` is never used (None), and the graph parameters get None when no offsets were
    drawn (``graph_augmentation.py:141-147`` returns zeros without touching them).  Parameter
    gradients leave as one flat tensor per pack (see ``_ParamPack``), written in place by the
    backward's reduce kernel."""

    @staticmethod
    def forward(ctx, x, desc, weights, keep, fire, want_attn, active, core, graph, tok_core, tok_graph,
                tensors=None):
        ws = S.workspace(desc, x.device)   # kept: the backward reuses its update field
        out, attn = S.step(desc, weights, x, fire=fire, want_attention=want_attn, ws=ws, active=active)
        if attn is not None:
            ctx.mark_non_differentiable(attn)
        ctx.save_for_backward(x)
        ctx.desc, ctx.weights, ctx.keep, ctx.fire = desc, weights, keep, fire
        ctx.ws = ws
        ctx.active = active
        ctx.packs = (core, graph)
        # the weights are passed to the kernels as raw pointers (not saved tensors), so autograd's
        # version check would not see an in-place update between forward and backward (an
        # optimizer step, load_state_dict, EMA swap): record the versions and check them ourselves
        ctx.versions = tuple((t, t._version) for t in (tensors or {}).values())
        return out, attn

    @staticmethod
    def backward(ctx, gout, gattn):
        (x,) = ctx.saved_tensors
        for t, v in ctx.versions:
            if t._version != v:
                raise RuntimeError(
                    "one of the variables needed for gradient computation has been modified by an "
                    f"inplace operation: a step weight of shape {tuple(t.shape)} is at version "
                    f"{t._version}; expected version {v} instead")
        desc = ctx.desc
        no_graph_use = (desc.flags & L.GRAPH) and desc.num_offsets == 0
        want, views, flats = {}, {}, [None, None]
        for i, pack in enumerate(ctx.packs):
            if pack is None or not ctx.needs_input_grad[9 + i] or (i == 1 and no_graph_use):
                continue
            flats[i] = torch.empty(sum(pack.sizes), dtype=torch.float32, device=x.device)
            views.update(pack.views(flats[i]))
            want.update(zip(pack.names, pack.params))
        gx, _ = S.step_backward(desc, ctx.weights, x, gout.contiguous(), fire=ctx.fire, want=want,
                                saved=ctx.ws, active=ctx.active, out=views)
        ctx.ws = None
        return (gx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, None, None,
                flats[0], flats[1], None)


def apply_step(model: nn.Module, x, desc, weights, keep, fire, want_attn=False, active=None, tensors=None):
    """One differentiable step: the HIP forward, and the HIP backward into the model's packs."""
    core, graph = param_packs(model, tensors)
    tc = core.token if core is not None else None
    tg = graph.token if graph is not None else None
    return _StepFn.apply(x, desc, weights, keep, fire, want_attn, active, core, graph, tc, tg, tensors)


def _step_tensors(model: nn.Module, graph) -> dict:
    """The step's weight tensors by short name, read straight from the modules' parameter dicts
    (``nn.Module.__getattr__`` costs ~1 us per attribute: building this dict through it was ~30 us
    of host time per step at the trainer's size, more than the step's kernels)."""
    mods = model._modules
    up = mods["update_net"]._modules
    l1, l2 = up["0"]._parameters, up["2"]._parameters
    t = {"perception": mods["perception"]._modules["conv"]._parameters["weight"],
         "w1": l1["weight"], "b1": l1["bias"], "w2": l2["weight"]}
    norm = mods["norm"]
    if isinstance(norm, nn.GroupNorm):
        t["gn_weight"] = norm._parameters["weight"]
        t["gn_bias"] = norm._parameters["bias"]
    if graph is not None:
        gm = graph._modules
        q, k, m = (gm[n]._parameters for n in ("query_proj", "key_proj", "msg_proj"))
        t.update(wq=q["weight"], bq=q["bias"], wk=k["weight"], bk=k["bias"], wm=m["weight"], bm=m["bias"],
                 scaling=graph._parameters["scaling"])
    return t


_DESC_TEMPLATES: dict = {}


def _step_desc(key, chosen, message_gain, fire_rate, fire_mode):
    """A fresh descriptor: the fields fixed by (shape, flags, model constants) copied from a cached
    template, then this call's offsets, message gain and fire fields (make_desc was ~10 us)."""
    tpl = _DESC_TEMPLATES.get(key)
    if tpl is None:
        B, C, H, W, hidden, d_model, flags, update_gain, alpha_thr, graph_thr, eps = key
        tpl = S.make_desc(B=B, C=C, H=H, W=W, hidden=hidden, d_model=d_model, offsets=[], flags=flags,
                          update_gain=update_gain, alpha_thr=alpha_thr, graph_alpha_thr=graph_thr,
                          message_gain=0.0, fire_rate=1.0, fire_mode=L.FIRE_NONE, gn_eps=eps)
        if len(_DESC_TEMPLATES) >= 256:
            _DESC_TEMPLATES.clear()
        _DESC_TEMPLATES[key] = tpl
    d = L.StepDesc.from_buffer_copy(tpl)
    if chosen:
        if len(chosen) > L.MAX_OFFSETS:
            raise ValueError(f"at most {L.MAX_OFFSETS} offsets per step (got {len(chosen)})")
        flat = [v for o in chosen for v in o]
        if min(flat) < -127 or max(flat) > 127:
            raise ValueError(f"offsets {chosen} out of int8 range")
        d.num_offsets = len(chosen)
        d.offsets[:len(flat)] = flat
    d.message_gain = float(message_gain)
    d.fire_rate = float(fire_rate)
    d.fire_mode = fire_mode
    return d


def run_step(model: nn.Module, x: torch.Tensor, fire_rate: float, graph, chosen, message_gain,
             hidden_only: bool, return_attention: bool, active=None):
    x = S.check_state(x, model.n_channels)
    B, C, H, W = x.shape
    flags = 0
    norm = model._modules["norm"]
    eps = 1e-3
    if isinstance(norm, nn.GroupNorm):
        if norm.num_groups != 1 or not norm.affine:
            raise ValueError("only GroupNorm(1, C, affine=True) is supported (ncagraph.py:68)")
        flags |= L.USE_GROUPNORM
        eps = norm.eps
    elif not isinstance(norm, nn.Identity):
        raise ValueError(f"unsupported norm module {type(norm).__name__}")
    tensors = _step_tensors(model, graph)
    d_model = 1
    graph_thr = None
    if graph is not None:
        flags |= graph.flags(return_attention)
        if hidden_only:
            flags |= L.HIDDEN_ONLY
        d_model = graph.d_model
        graph_thr = graph.alpha_thr
    # stochastic fire mask: the reference's torch.rand draw, on x.device (ncagraph.py:144-146)
    fire = None
    fire_mode = L.FIRE_NONE
    if fire_rate < 1.0:
        fire = torch.rand(B, 1, H, W, device=x.device)
        fire_mode = L.FIRE_RAND_F32
    alpha_thr = float(model.alpha_thr)
    key = (B, C, H, W, tensors["w1"].shape[0], d_model, flags, float(model.update_gain), alpha_thr,
           alpha_thr if graph_thr is None else float(graph_thr), float(eps))
    desc = _step_desc(key, chosen, message_gain, fire_rate, fire_mode)
    w, keep = S.make_weights(tensors)
    if torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in tensors.values())):
        out, attn = apply_step(model, x, desc, w, keep, fire, return_attention, active, tensors)
    else:
        out, attn = S.step(desc, w, x, fire=fire, want_attention=return_attention, active=active)
    return out, attn
