"""CPU oracle for the BACKWARD of the NCA step — TEST INFRASTRUCTURE ONLY.

The vector-Jacobian product of one step (BPTT through
``NeuralCAGraph.forward`` ``src/modules/ncagraph.py:106-168`` / ``NeuralCA.forward``
``src/modules/nca.py:64-105``), written out by hand in numpy from the forward restated in
``oracle/nca_oracle.py``.  Same rules as that module: only ``tests/`` (and ``bench.py``'s CPU
leg) may import it; the product path never does.

Parity pinning: ``tests/test_oracle_grad.py`` checks it against the reference's own autograd
(``tests/golden/grad_*.npz`` / ``bptt_*.npz``, made by ``tests/golden/make_golden_grad.py``), in
float64, to ~1e-12 relative.

What is differentiated, following the reference's graph of tensors:

* the alive masks (``max_pool > thr``) and the fire mask are constants (comparisons);
* the perception weight is frozen (``perception.py:19``) and ``gate_mlp`` is never called, so
  neither gets a gradient;
* in torus mode the offset weights are mathematically constant (mean(roll K) = mean K), so the
  Q/K/scaling gradients are exactly zero here; the reference's float32 autograd returns rounding
  noise of ~1e-7 for them (visible in the fixtures).
"""
from __future__ import annotations

import numpy as np

from .nca_oracle import alive_mask, conv1x1, perceive, shift_pad, shift_roll


def _shift_adj(z: np.ndarray, dy: int, dx: int, zero_pad: bool) -> np.ndarray:
    """Adjoint of the reference shift (graph_augmentation.py:85-97): roll back, or for the
    row-only zero-padded shift, shift rows the other way (zeros fill)."""
    if zero_pad:
        return shift_pad(z, -dy, 0)
    return np.roll(z, (-dy, -dx), axis=(2, 3))


def perceive_adj(gy: np.ndarray, weight: np.ndarray) -> np.ndarray:
    """Adjoint of ``perceive`` (perception.py:21-26): the transposed depthwise 3x3 correlation,
    zero padding, through the [3,C] feature reorder."""
    B, C3, H, W = gy.shape
    C = C3 // 3
    w = weight.reshape(C, 3, 3, 3).astype(gy.dtype)       # [c, f, a, b]
    g = gy.reshape(B, 3, C, H, W)
    gp = np.zeros((B, C, H + 2, W + 2), gy.dtype)
    for a in range(3):
        for b in range(3):
            for f in range(3):
                # y(i,j) += w[a,b] x(i+a-1, j+b-1)  =>  gx(i+a-1, j+b-1) += w[a,b] gy(i,j)
                gp[:, :, a:a + H, b:b + W] += g[:, f] * w[None, :, f, a, b, None, None]
    return gp[:, :, 1:-1, 1:-1]


def _sum_outer(g: np.ndarray, z: np.ndarray) -> np.ndarray:
    """sum over (b,h,w) of g[:,o] z[:,i] -> [O, I] (a 1x1-conv weight gradient)."""
    return np.einsum("bohw,bihw->oi", g, z, optimize=True)


def nca_step_vjp(x: np.ndarray, p: dict, cfg: dict, gy: np.ndarray, *, chosen=None, fire_mask=None):
    """Gradients of ``sum(nca_step(x) * gy)`` w.r.t. ``x`` and the trainable parameters.

    Returns ``(gx, grads)``; ``grads`` maps state_dict keys to arrays of the parameter's shape.
    Keys of parameters the reference leaves without a gradient are absent (no graph call, or
    no offsets drawn).
    """
    dt = x.dtype
    B, C, H, W = x.shape
    HW = H * W
    f64 = lambda k: np.asarray(p[k], dt)  # noqa: E731
    W1 = f64("update_net.0.weight").reshape(-1, 3 * C)
    b1 = f64("update_net.0.bias")
    W2 = f64("update_net.2.weight").reshape(C, -1)
    graph = cfg.get("graph", True)
    use_gn = cfg.get("use_groupnorm", True)
    chosen = list(chosen or [])
    zp = bool(cfg.get("zero_padded_shift", False))
    shift = shift_pad if zp else shift_roll

    # ---------------- forward, keeping what the backward needs (nca_oracle.nca_step) -------
    y = perceive(x, p["perception.conv.weight"])
    hpre = conv1x1(y, W1, b1)
    h = np.maximum(hpre, 0)
    dl = conv1x1(h, W2, None)
    dxa = dl
    msg_terms = None
    if graph and chosen:
        Wq, bq = f64("graph.query_proj.weight").reshape(-1, C), f64("graph.query_proj.bias")
        Wk, bk = f64("graph.key_proj.weight").reshape(-1, C), f64("graph.key_proj.bias")
        Wm, bm = f64("graph.msg_proj.weight").reshape(C, C), f64("graph.msg_proj.bias")
        Q, Kf, M = conv1x1(x, Wq, bq), conv1x1(x, Wk, bk), conv1x1(x, Wm, bm)
        qp = Q.mean(axis=(2, 3))
        a2a = cfg["alive_to_alive"]
        A_send = alive_mask(x, cfg["alpha_thr"]) if a2a else None
        msgs, kps, sends = [], [], []
        for dy, dx in chosen:
            Ms = shift(M, dy, dx)
            As = shift(A_send, dy, dx) if a2a else None
            msgs.append(Ms * As if a2a else Ms)
            sends.append(As)
            kps.append(shift(Kf, dy, dx).mean(axis=(2, 3)))
        L = np.stack([(qp * kp).sum(1) for kp in kps], 0)              # [N,B]
        Ls = L - L.max(axis=0, keepdims=True)
        s = np.asarray(p["graph.scaling"], dt)
        denom = np.abs(s) + dt.type(1e-6)
        e = np.exp(Ls / denom)
        Wt = e / e.sum(axis=0, keepdims=True)                          # [N,B]
        agg = (np.stack(msgs, 0) * Wt[:, :, None, None, None]).sum(0)
        m = agg.copy()
        if cfg["hidden_only"] and C >= 4:
            m[:, :4] = 0
        tm = np.tanh(m)
        dxa = dl + tm * dt.type(cfg["message_gain"])
        msg_terms = (Wq, Wk, Wm, Q, qp, kps, msgs, sends, Ls, Wt, denom, s, tm)
    fire = np.ones((B, 1, H, W), dt) if fire_mask is None else fire_mask.astype(dt)
    A_pre = alive_mask(x, cfg["alpha_thr"])
    dxb = dxa * fire * A_pre
    if use_gn:
        flat = dxb.reshape(B, -1)
        mu = flat.mean(1)[:, None, None, None]
        rstd = (1.0 / np.sqrt(flat.var(1) + dt.type(1e-3)))[:, None, None, None]
        xhat = (dxb - mu) * rstd
        gam = f64("norm.weight")[None, :, None, None]
        xn = xhat * gam + f64("norm.bias")[None, :, None, None]
    else:
        xn = dxb
    t = np.tanh(xn)
    xt = x + t * dt.type(cfg["update_gain"])
    post = alive_mask(xt, cfg["alpha_thr"])

    # ---------------- backward ----------------------------------------------------------
    grads = {}
    g_xt = gy.astype(dt).copy()
    g_xt[:, 3:4] *= post                                                # (:158-166)
    gx = g_xt.copy()                                                    # residual x + ...
    g_xn = g_xt * dt.type(cfg["update_gain"]) * (1 - t * t)             # (:154)
    if use_gn:                                                          # (:153) GroupNorm(1,C)
        grads["norm.weight"] = (g_xn * xhat).sum(axis=(0, 2, 3))
        grads["norm.bias"] = g_xn.sum(axis=(0, 2, 3))
        u = g_xn * gam
        mu_u = u.reshape(B, -1).mean(1)[:, None, None, None]
        mu_ux = (u * xhat).reshape(B, -1).mean(1)[:, None, None, None]
        g_dxb = rstd * (u - mu_u - xhat * mu_ux)
    else:
        g_dxb = g_xn
    g_dxa = g_dxb * fire * A_pre                                        # (:144-150)
    # local update path: dl = W2 relu(W1 y + b1)                        # (:128-131)
    grads["update_net.2.weight"] = _sum_outer(g_dxa, h).reshape(p["update_net.2.weight"].shape)
    g_h = conv1x1(g_dxa, W2.T, None)
    g_hpre = g_h * (hpre > 0)
    grads["update_net.0.weight"] = _sum_outer(g_hpre, y).reshape(p["update_net.0.weight"].shape)
    grads["update_net.0.bias"] = g_hpre.sum(axis=(0, 2, 3))
    gx += perceive_adj(conv1x1(g_hpre, W1.T, None), p["perception.conv.weight"])
    if msg_terms is not None:                                           # graph_augmentation.py:104-169
        Wq, Wk, Wm, Q, qp, kps, msgs, sends, Ls, Wt, denom, s, tm = msg_terms
        g_m = g_dxa * dt.type(cfg["message_gain"]) * (1 - tm * tm)      # (ncagraph.py:98-103)
        if cfg["hidden_only"] and C >= 4:
            g_m[:, :4] = 0
        g_M = np.zeros_like(x)
        g_W = np.zeros_like(Wt)                                         # [N,B]
        for o, (dy, dx) in enumerate(chosen):
            g_W[o] = (g_m * msgs[o]).sum(axis=(1, 2, 3))
            g_ms = g_m * Wt[o][:, None, None, None]
            if sends[o] is not None:
                g_ms = g_ms * sends[o]
            g_M += _shift_adj(g_ms, dy, dx, zp)
        grads["graph.msg_proj.weight"] = _sum_outer(g_M, x).reshape(p["graph.msg_proj.weight"].shape)
        grads["graph.msg_proj.bias"] = g_M.sum(axis=(0, 2, 3))
        gx += conv1x1(g_M, Wm.T, None)
        if zp:
            # softmax over offsets with temperature |scaling| + 1e-6 (graph_augmentation.py:150-154)
            g_z = Wt * (g_W - (Wt * g_W).sum(0, keepdims=True))             # [N,B]
            g_L = g_z / denom
            g_denom = -(g_z * Ls).sum() / (denom * denom)
            g_s = np.asarray(g_denom * np.sign(s), dt)
            g_qp = sum(g_L[o][:, None] * kps[o] for o in range(len(chosen)))   # [B,d]  (:114,:131)
            d = qp.shape[1]
            g_K = np.zeros((B, d, H, W), dt)
            for o, (dy, dx) in enumerate(chosen):
                g_kp = (g_L[o][:, None] * qp)[:, :, None, None] / HW
                g_K += _shift_adj(np.broadcast_to(g_kp, (B, d, H, W)).copy(), dy, dx, zp)
            g_Q = np.broadcast_to(g_qp[:, :, None, None] / HW, (B, d, H, W))
            gx += conv1x1(g_Q, Wq.T, None) + conv1x1(g_K, Wk.T, None)
        else:
            # torus: the offset weights do not depend on Q/K/scaling at all (see header)
            d = Q.shape[1]
            g_Q = g_K = np.zeros((B, d, H, W), dt)
            g_s = np.zeros((), dt)
        grads["graph.scaling"] = g_s.reshape(np.shape(p["graph.scaling"]))
        grads["graph.query_proj.weight"] = _sum_outer(g_Q, x).reshape(p["graph.query_proj.weight"].shape)
        grads["graph.query_proj.bias"] = g_Q.sum(axis=(0, 2, 3))
        grads["graph.key_proj.weight"] = _sum_outer(g_K, x).reshape(p["graph.key_proj.weight"].shape)
        grads["graph.key_proj.bias"] = g_K.sum(axis=(0, 2, 3))
    return gx, grads
