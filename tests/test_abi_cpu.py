"""CPU-side checks of the C ABI: the library loads, exports every symbol include/gnca.h declares,
the ctypes mirrors match the C struct layout, and host-only entry points behave (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from graph_neural_cellular_automata_amd import _lib as L
from graph_neural_cellular_automata_amd import step as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gnca.h")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(L.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return L.load()


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(gnca_\w+)\s*\(", src, re.M)))


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert set(names) == set(L.EXPORTS), names
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", out, re.M), f"{n} not exported"
        assert hasattr(lib, n)


def test_abi_version(lib):
    assert lib.gnca_abi_version() == L.ABI_VERSION
    assert lib.gnca_status_string(0) == b"ok"


def test_struct_layout_matches_header(tmp_path):
    """Compile a C probe against gnca.h and compare offsetof/sizeof with the ctypes mirrors."""
    fields_d = [f for f, _ in L.StepDesc._fields_]
    fields_w = [f for f, _ in L.Weights._fields_]
    fields_g = [f for f, _ in L.Grads._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "gnca.h"', 'int main(void){']
    lines.append('printf("desc %zu\\n", sizeof(gnca_step_desc));')
    lines.append('printf("weights %zu\\n", sizeof(gnca_weights));')
    lines.append('printf("grads %zu\\n", sizeof(gnca_grads));')
    for f in fields_g:
        lines.append(f'printf("g.{f} %zu\\n", offsetof(gnca_grads, {f}));')
    for f in fields_d:
        lines.append(f'printf("d.{f} %zu\\n", offsetof(gnca_step_desc, {f}));')
    for f in fields_w:
        lines.append(f'printf("w.{f} %zu\\n", offsetof(gnca_weights, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    assert int(got["desc"]) == ctypes.sizeof(L.StepDesc)
    assert int(got["weights"]) == ctypes.sizeof(L.Weights)
    for f in fields_d:
        assert int(got[f"d.{f}"]) == getattr(L.StepDesc, f).offset, f
    for f in fields_w:
        assert int(got[f"w.{f}"]) == getattr(L.Weights, f).offset, f
    assert int(got["grads"]) == ctypes.sizeof(L.Grads)
    for f in fields_g:
        assert int(got[f"g.{f}"]) == getattr(L.Grads, f).offset, f


def _desc(**kw):
    base = dict(B=4, C=16, H=72, W=72, hidden=128, d_model=16, offsets=[(2, 3), (-4, 1)],
                flags=L.GRAPH | L.USE_GROUPNORM | L.ALIVE_TO_ALIVE | L.HIDDEN_ONLY,
                update_gain=0.05, alpha_thr=0.12, message_gain=0.25, fire_rate=0.5,
                fire_mode=L.FIRE_HASH)
    base.update(kw)
    return S.make_desc(**base)


def test_workspace_bytes_host_only(lib):
    d = _desc()
    n = lib.gnca_workspace_bytes(ctypes.byref(d))
    # at least the dx buffer (B*C*H*W fp32)
    assert n >= 4 * 16 * 72 * 72 * 4
    d2 = _desc(B=8)
    assert lib.gnca_workspace_bytes(ctypes.byref(d2)) > n


@pytest.mark.parametrize("bad", [dict(C=3), dict(C=36), dict(hidden=512), dict(B=0), dict(H=0)])
def test_workspace_bytes_rejects_unsupported(lib, bad):
    d = _desc(**bad)
    assert lib.gnca_workspace_bytes(ctypes.byref(d)) == 0


def test_step_rejects_bad_args_without_touching_gpu(lib):
    d = _desc()
    w = L.Weights()
    # null pointers are rejected before any launch
    rc = lib.gnca_step_f32(ctypes.byref(d), ctypes.byref(w), None, None, None, None, None, 0, None)
    assert rc == -1
    rc = lib.gnca_rollout_f32(ctypes.byref(d), ctypes.byref(w), 3, None, None, None, None, None, 0, None)
    assert rc == -1


def test_bwd_workspace_bytes_host_only(lib):
    d = _desc()
    n = lib.gnca_bwd_workspace_bytes(ctypes.byref(d))
    # forward workspace + U + dY(3C) + dG at least
    assert n >= lib.gnca_workspace_bytes(ctypes.byref(d)) + 5 * 4 * 16 * 72 * 72 * 4
    for bad in (dict(C=3), dict(C=36), dict(hidden=512), dict(B=0)):
        assert lib.gnca_bwd_workspace_bytes(ctypes.byref(_desc(**bad))) == 0


def test_bwd_rejects_bad_args_without_touching_gpu(lib):
    d = _desc()
    w = L.Weights()
    g = L.Grads()
    rc = lib.gnca_step_bwd_f32(ctypes.byref(d), ctypes.byref(w), None, None, None, None, None,
                               ctypes.byref(g), None, None, 0, None)
    rc2 = lib.gnca_step_masked_f32(ctypes.byref(d), ctypes.byref(w), None, None, None, None, None, 0, None)
    assert rc2 == -1
    assert rc == -1


def test_k1_variant_names(lib):
    """gnca_k1_variant (host-only) names the K1 each BASELINE workload shape plans: the bf16-split
    kernels for 16 and 32 channels, the fp32-MFMA kernel for other shape classes."""
    from graph_neural_cellular_automata_amd import _lib as L_
    flags = L_.USE_GROUPNORM | L_.GRAPH | L_.HIDDEN_ONLY | L_.ALIVE_TO_ALIVE

    def name(B, C, H, offs, hidden=128, graph=True):
        d = S.make_desc(B=B, C=C, H=H, W=H, hidden=hidden, d_model=16, offsets=offs,
                        flags=flags if graph else L_.USE_GROUPNORM, update_gain=0.05, alpha_thr=0.12,
                        message_gain=0.25, fire_rate=0.5, fire_mode=L_.FIRE_HASH)
        return S.k1_variant(d)

    r4 = [(dy, dx) for dy in range(-4, 5) for dx in range(-4, 5) if max(abs(dy), abs(dx)) > 1][:8]
    r5 = [(dy, dx) for dy in range(-5, 6) for dx in range(-5, 6) if max(abs(dy), abs(dx)) > 1][:16]
    assert name(1024, 16, 72, r4) == ("gnca_k1_split<24,36,4,4,8>", "bf16x6")
    assert name(8, 16, 72, r4) == ("gnca_k1_split<8,24,4,4,8>", "bf16x6")
    assert name(8, 16, 72, [], graph=False) == ("gnca_k1_split<8,24,1,4,0>", "bf16x6")
    # classic steps at large batches (and the trainers' message-off graph steps): 24x36 tiles
    assert name(128, 16, 72, [], graph=False) == ("gnca_k1_split<24,36,1,4,0>", "bf16x6")
    d_off = S.make_desc(B=128, C=16, H=72, W=72, hidden=128, d_model=16, offsets=r4, flags=flags,
                        update_gain=0.05, alpha_thr=0.12, message_gain=0.0, fire_rate=0.5,
                        fire_mode=L_.FIRE_HASH)
    assert S.k1_variant(d_off) == ("gnca_k1_split<24,36,1,4,0>", "bf16x6")
    assert name(128, 32, 128, r5) == ("gnca_k1_split32<16,16,5,8,16>", "bf16x6")
    # the rollout's compact update field: large batches on the bf16-split K1s only
    comp = lambda B, C, H, offs, graph=True: S.rollout_compact(S.make_desc(
        B=B, C=C, H=H, W=H, hidden=128, d_model=16, offsets=offs,
        flags=flags if graph else L_.USE_GROUPNORM, update_gain=0.05, alpha_thr=0.12,
        message_gain=0.25, fire_rate=0.5, fire_mode=L_.FIRE_HASH))
    assert comp(1024, 16, 72, r4) and comp(1024, 16, 72, [], graph=False)
    assert not comp(8, 16, 72, r4) and comp(128, 32, 128, r5) and not comp(4, 32, 128, r5)
    nm, ar = name(4, 12, 20, r4, hidden=64)
    assert nm.startswith("gnca_k1_update<12,64,") and ar == "f32"
    buf = ctypes.create_string_buffer(8)
    assert lib.gnca_k1_variant(None, buf, 8, None) != 0


def test_bb_variant_names(lib):
    """gnca_bb_variant (host-only) names the backward MLP kernel each training shape plans: the
    lean-layout 24x24 instances once a 72^2 batch fills the chip (B >= 96), 8x24 below (B >= 8), the
    graph (K = 8) and the classic / message-off (K = 0) instances, the runtime-geometry kernel
    elsewhere."""
    from graph_neural_cellular_automata_amd import _lib as L_
    flags = L_.USE_GROUPNORM | L_.GRAPH | L_.HIDDEN_ONLY | L_.ALIVE_TO_ALIVE
    r4 = [(dy, dx) for dy in range(-4, 5) for dx in range(-4, 5) if max(abs(dy), abs(dx)) > 1][:8]

    def name(B, H, offs, graph=True, gain=0.25, C=16):
        d = S.make_desc(B=B, C=C, H=H, W=H, hidden=128, d_model=16, offsets=offs,
                        flags=flags if graph else L_.USE_GROUPNORM, update_gain=0.05, alpha_thr=0.12,
                        message_gain=gain, fire_rate=0.5, fire_mode=L_.FIRE_HASH)
        return S.bb_variant(d)

    assert name(1024, 72, r4) == "gnca_b_mlp<16,128,1,24,24,4,4,8,1>"
    assert name(128, 72, r4) == "gnca_b_mlp<16,128,1,24,24,4,4,8,1>"
    assert name(96, 72, r4) == "gnca_b_mlp<16,128,1,24,24,4,4,8,1>"
    assert name(128, 72, r4, gain=0.0) == "gnca_b_mlp<16,128,1,24,24,1,4,0,1>"
    assert name(128, 72, [], graph=False) == "gnca_b_mlp<16,128,1,24,24,1,4,0,1>"
    assert name(64, 72, r4) == "gnca_b_mlp<16,128,1,8,24,4,4,8,0>"
    assert name(8, 72, r4) == "gnca_b_mlp<16,128,1,8,24,4,4,8,0>"
    assert name(2, 72, r4) == "gnca_b_mlp<16,128,1,0,0,0,0,-1,0>"   # smaller tiles, runtime geometry
    assert name(16, 40, r4) == "gnca_b_mlp<16,128,1,8,16,4,4,8,0>"
    assert name(16, 40, r4, C=12).startswith("gnca_b_mlp<12,")
    buf = ctypes.create_string_buffer(8)
    assert lib.gnca_bb_variant(None, buf, 8) != 0
