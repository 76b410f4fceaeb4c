"""Shared forward of NeuralCA / NeuralCAGraph: descriptor + weights -> one HIP step."""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import _lib as L
from .. import step as S


class _StepFn(torch.autograd.Function):
    """The HIP step as an autograd node (BPTT through the trainers' rollouts).

    Forward: ``gnca_step_f32`` into a workspace that the node keeps (the step's update field and
    GroupNorm partials, ~one state of memory).  Backward: ``gnca_step_bwd_f32`` on that saved
    workspace; everything else (perception, hidden layer, message) is recomputed from the input
    state, so a rollout keeps two state-sized tensors per step alive, far less than the
    reference's per-op activations.  Gradients follow the
    reference's graph of tensors: masks are constants, the perception weight is frozen,
    ``gate_mlp`` is never used (None), and the graph parameters get None when no offsets were
    drawn (``graph_augmentation.py:141-147`` returns zeros without touching them)."""

    @staticmethod
    def forward(ctx, x, desc, weights, keep, fire, want_attn, names, active, *params):
        ws = S.workspace(desc, x.device)   # kept: the backward reuses its update field
        out, attn = S.step(desc, weights, x, fire=fire, want_attention=want_attn, ws=ws, active=active)
        if attn is not None:
            ctx.mark_non_differentiable(attn)
        ctx.save_for_backward(x)
        ctx.desc, ctx.weights, ctx.keep, ctx.fire, ctx.names = desc, weights, keep, fire, names
        ctx.ws = ws
        ctx.active = active
        ctx.params = params
        return out, attn

    @staticmethod
    def backward(ctx, gout, gattn):
        (x,) = ctx.saved_tensors
        desc = ctx.desc
        no_graph_use = (desc.flags & L.GRAPH) and desc.num_offsets == 0
        need = ctx.needs_input_grad[8:]
        want = {}
        for name, p, nd in zip(ctx.names, ctx.params, need):
            if not nd or name not in S.GRAD_FIELDS:
                continue
            if no_graph_use and name.startswith("graph."):
                continue
            want[name] = p
        gx, grads = S.step_backward(desc, ctx.weights, x, gout.contiguous(), fire=ctx.fire, want=want,
                                    saved=ctx.ws, active=ctx.active)
        ctx.ws = None
        pgrads = [grads.get(n) for n in ctx.names]
        return (gx if ctx.needs_input_grad[0] else None, None, None, None, None, None, None, None,
                *pgrads)


def run_step(model: nn.Module, x: torch.Tensor, fire_rate: float, graph, chosen, message_gain,
             hidden_only: bool, return_attention: bool, active=None):
    x = S.check_state(x, model.n_channels)
    B, C, H, W = x.shape
    flags = 0
    norm = model.norm
    eps = 1e-3
    if isinstance(norm, nn.GroupNorm):
        if norm.num_groups != 1 or not norm.affine:
            raise ValueError("only GroupNorm(1, C, affine=True) is supported (ncagraph.py:68)")
        flags |= L.USE_GROUPNORM
        eps = norm.eps
    elif not isinstance(norm, nn.Identity):
        raise ValueError(f"unsupported norm module {type(norm).__name__}")
    tensors = dict(perception=model.perception.conv.weight, w1=model.update_net[0].weight,
                   b1=model.update_net[0].bias, w2=model.update_net[2].weight)
    if flags & L.USE_GROUPNORM:
        tensors.update(gn_weight=norm.weight, gn_bias=norm.bias)
    d_model = 1
    graph_thr = None
    if graph is not None:
        flags |= graph.flags(return_attention)
        if hidden_only:
            flags |= L.HIDDEN_ONLY
        tensors.update(graph.weight_tensors())
        d_model = graph.d_model
        graph_thr = graph.alpha_thr
    # stochastic fire mask: the reference's torch.rand draw, on x.device (ncagraph.py:144-146)
    fire = None
    fire_mode = L.FIRE_NONE
    if fire_rate < 1.0:
        fire = torch.rand(B, 1, H, W, device=x.device)
        fire_mode = L.FIRE_RAND_F32
    desc = S.make_desc(B=B, C=C, H=H, W=W, hidden=model.update_net[0].out_channels,
                       d_model=d_model, offsets=chosen or [], flags=flags,
                       update_gain=model.update_gain, alpha_thr=model.alpha_thr,
                       graph_alpha_thr=graph_thr, message_gain=message_gain,
                       fire_rate=fire_rate, fire_mode=fire_mode, gn_eps=eps)
    w, keep = S.make_weights(tensors)
    named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
    if torch.is_grad_enabled() and (x.requires_grad or named):
        names = tuple(n for n, _ in named)
        params = [p for _, p in named]
        out, attn = _StepFn.apply(x, desc, w, keep, fire, return_attention, names, active, *params)
    else:
        out, attn = S.step(desc, w, x, fire=fire, want_attention=return_attention, active=active)
    return out, attn
