"""The parameter-pack routing of the step's autograd node (modules/_stepper.py), on the CPU with a
stand-in step: per-step flat gradients summed by autograd land in the right parameters with the
right shapes; packs the steps never feed keep grad=None (the reference's None for unused graph
parameters and for gate_mlp); the cached token survives an optimiser step."""
import torch

from graph_neural_cellular_automata_amd import NeuralCAGraph
from graph_neural_cellular_automata_amd.modules._stepper import param_packs


class _FakeStep(torch.autograd.Function):
    """y = x; d tok_core = c * ones, d tok_graph = g * ones (or None when g is None)."""

    @staticmethod
    def forward(ctx, x, c, g, tc, tg):
        ctx.c, ctx.g, ctx.n = c, g, (tc.numel(), tg.numel())
        return x.clone()

    @staticmethod
    def backward(ctx, gy):
        fg = None if ctx.g is None else torch.full((ctx.n[1],), float(ctx.g))
        return gy, None, None, torch.full((ctx.n[0],), float(ctx.c)), fg


def _run(m, gs):
    core, graph = param_packs(m)
    x = torch.ones(3, requires_grad=True)
    y = x
    for i, g in enumerate(gs):
        y = _FakeStep.apply(y, i + 1, g, core.token, graph.token)
    y.sum().backward()
    return core, graph


def test_pack_routes_and_sums():
    m = NeuralCAGraph(8, update_hidden=16)
    core, graph = _run(m, [None, 2.0, 5.0])
    assert "update_net.0.weight" in core.names and "graph.msg_proj.weight" in graph.names
    assert not any("gate_mlp" in n for n in core.names + graph.names)
    params = dict(m.named_parameters())
    for n in core.names:
        assert params[n].grad.shape == params[n].shape
        assert torch.equal(params[n].grad, torch.full_like(params[n], 6.0))   # 1 + 2 + 3
    for n in graph.names:
        assert torch.equal(params[n].grad, torch.full_like(params[n], 7.0))   # None + 2 + 5
    assert all(p.grad is None for n, p in params.items() if "gate_mlp" in n)


def test_unused_graph_pack_keeps_none_and_token_is_cached():
    m = NeuralCAGraph(8, update_hidden=16)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    core, graph = _run(m, [None, None])
    params = dict(m.named_parameters())
    assert all(params[n].grad is None for n in graph.names)
    assert torch.equal(params["norm.weight"].grad, torch.full_like(params["norm.weight"], 3.0))
    opt.step()
    opt.zero_grad(set_to_none=True)
    core2, graph2 = _run(m, [1.0])
    assert core2 is core and graph2 is graph
    assert torch.equal(params["norm.bias"].grad, torch.full_like(params["norm.bias"], 1.0))
    assert torch.equal(params["graph.scaling"].grad, torch.full_like(params["graph.scaling"], 1.0))


def test_frozen_model_has_no_packs_twice():
    """All parameters frozen (input-gradient / saliency BPTT): no packs, and the cached empty
    entry must not break the second step (IndexError on the cache check)."""
    m = NeuralCAGraph(8, update_hidden=16)
    m.requires_grad_(False)
    assert param_packs(m) == (None, None)
    assert param_packs(m) == (None, None)
    m.requires_grad_(True)
    core, graph = param_packs(m)
    assert core is not None and graph is not None


def test_loss_rejects_mismatched_target():
    """The fused loss validates the target against pred before any device work (the reference's
    F.mse_loss raises on a shape it cannot broadcast)."""
    import pytest
    from graph_neural_cellular_automata_amd.loss import loss_premult_rgba
    pred = torch.zeros(3, 4, 8, 8)
    for bad in (torch.zeros(3, 3, 8, 8), torch.zeros(3, 4, 8, 9), torch.zeros(2, 4, 8, 8),
                torch.zeros(4, 7, 8), torch.zeros(8, 8)):
        with pytest.raises(ValueError, match="does not match pred"):
            loss_premult_rgba(pred, bad)
    for ok in (torch.zeros(4, 8, 8), torch.zeros(1, 4, 8, 8), torch.zeros(3, 4, 8, 8)):
        with pytest.raises(RuntimeError, match="no CPU path"):   # shape accepted, then no CPU path
            loss_premult_rgba(pred, ok)


def test_param_packs_fast_path_and_deepcopy():
    """The packs' fast-path cache (weight-tensor identities + requires_grad flags) returns the
    same packs for the same parameters, rebuilds when a flag changes, and leaves the module
    deep-copyable (the cache is a side table, not a module attribute)."""
    import copy

    from graph_neural_cellular_automata_amd import NeuralCAGraph
    from graph_neural_cellular_automata_amd.modules._stepper import _step_tensors, param_packs
    m = NeuralCAGraph(16, 64)
    a = param_packs(m, _step_tensors(m, m.graph))
    assert param_packs(m, _step_tensors(m, m.graph)) is a
    m.update_net[0].weight.requires_grad_(False)
    c = param_packs(m, _step_tensors(m, m.graph))
    assert c is not a and "update_net.0.weight" not in c[0].names
    m2 = copy.deepcopy(m)
    assert param_packs(m2, _step_tensors(m2, m2.graph)) is not c
