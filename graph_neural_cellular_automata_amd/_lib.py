"""ctypes binding of libgnca.so (include/gnca.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950) and
loaded from this package directory.  There is no fallback: if the library is missing or does
not match the ABI version, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  — load torch's HIP runtime first; libgnca.so binds to it by soname

_HERE = os.path.dirname(os.path.abspath(__file__))
# GNCA_LIB_PATH: an alternative build of the same library (A/B measurement runs only)
LIB_PATH = os.environ.get("GNCA_LIB_PATH") or os.path.join(_HERE, "libgnca.so")

ABI_VERSION = 2
MAX_OFFSETS = 128

GRAPH = 1 << 0
USE_GROUPNORM = 1 << 1
HIDDEN_ONLY = 1 << 2
ALIVE_TO_ALIVE = 1 << 3
ZERO_PAD_SHIFT = 1 << 4
ATTENTION = 1 << 5

FIRE_NONE = 0
FIRE_RAND_F32 = 1
FIRE_MASK_U8 = 2
FIRE_HASH = 3


class StepDesc(ctypes.Structure):
    """Mirror of gnca_step_desc (include/gnca.h)."""
    _fields_ = [
        ("B", ctypes.c_int32), ("C", ctypes.c_int32), ("H", ctypes.c_int32), ("W", ctypes.c_int32),
        ("hidden", ctypes.c_int32), ("d_model", ctypes.c_int32), ("num_offsets", ctypes.c_int32),
        ("fire_mode", ctypes.c_int32), ("flags", ctypes.c_uint32),
        ("update_gain", ctypes.c_float), ("alpha_thr", ctypes.c_float),
        ("graph_alpha_thr", ctypes.c_float),
        ("message_gain", ctypes.c_float), ("gn_eps", ctypes.c_float), ("fire_rate", ctypes.c_float),
        ("rng_seed", ctypes.c_uint64), ("rng_step", ctypes.c_int64), ("sample_base", ctypes.c_int64),
        ("offsets", ctypes.c_int8 * (2 * MAX_OFFSETS)),
    ]


class Weights(ctypes.Structure):
    """Mirror of gnca_weights (include/gnca.h): device pointers in reference layouts."""
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "perception", "w1", "b1", "w2", "gn_weight", "gn_bias",
        "wq", "bq", "wk", "bk", "wm", "bm", "scaling")]


class Grads(ctypes.Structure):
    """Mirror of gnca_grads (include/gnca.h): device output pointers in reference layouts."""
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "w1", "b1", "w2", "gn_weight", "gn_bias", "wq", "bq", "wk", "bk", "wm", "bm", "scaling")]


class DamageDesc(ctypes.Structure):
    """Mirror of gnca_damage_desc (include/gnca.h)."""
    _fields_ = [("B", ctypes.c_int32), ("C", ctypes.c_int32), ("H", ctypes.c_int32), ("W", ctypes.c_int32),
                ("kind", ctypes.c_int32), ("size", ctypes.c_int32), ("p", ctypes.c_float),
                ("alpha_thr", ctypes.c_float), ("softness", ctypes.c_float), ("sigma", ctypes.c_float)]


DMG_SQUARE, DMG_CIRCLE, DMG_STRIPE_H, DMG_STRIPE_V = 0, 1, 2, 3
DMG_ALPHA_DROP, DMG_ALPHA_DROP_SOFT, DMG_SALT_PEPPER, DMG_GAUSSIAN, DMG_HIDDEN_NOISE = 4, 5, 6, 7, 8

EXPORTS = ("gnca_abi_version", "gnca_status_string", "gnca_last_hip_error",
           "gnca_workspace_bytes", "gnca_step_f32", "gnca_step_phases_f32", "gnca_message_f32",
           "gnca_perceive_f32", "gnca_rollout_f32", "gnca_bwd_workspace_bytes", "gnca_step_bwd_f32",
           "gnca_fire_mask_u8", "gnca_step_masked_f32", "gnca_damage_f32", "gnca_loss_premult_f32",
           "gnca_loss_premult_bwd_f32", "gnca_k1_variant", "gnca_rollout_stamped_f32",
           "gnca_rollout_ex_f32", "gnca_bb_variant")

PHASE_K0, PHASE_K1, PHASE_K2 = 1, 2, 4
PHASE_ALL = 7
PHASE_ALIVE = 8   # rollout mode: K2 hands the next step's alive masks to K1 (include/gnca.h)
ROLLOUT_ALIVE_IN, ROLLOUT_ALIVE_OUT = 1, 2   # gnca_rollout_ex_f32 pieces (include/gnca.h)
ROLLOUT_PENDING_IN, ROLLOUT_PENDING_OUT = 4, 8   # fold rollouts: the last step handed over unfinished
ROLLOUT_FOLD = 16   # request the fold on the compact field too (include/gnca.h)
PHASE_COMPACT = 16   # rollout mode: K1 packs the live cells' dx per tile, K2 unpacks (include/gnca.h)

_lib = None


class GncaError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libgnca.so (raises if absent or ABI-mismatched — there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GncaError(
            f"libgnca.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950). The NCA step has no CPU fallback.")
    lib = ctypes.CDLL(path)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.gnca_abi_version.restype = ctypes.c_int
    lib.gnca_status_string.restype = ctypes.c_char_p
    lib.gnca_status_string.argtypes = [ctypes.c_int]
    lib.gnca_last_hip_error.restype = ctypes.c_int
    lib.gnca_workspace_bytes.restype = sz
    lib.gnca_workspace_bytes.argtypes = [ctypes.POINTER(StepDesc)]
    lib.gnca_step_f32.restype = ctypes.c_int
    lib.gnca_step_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights), vp, vp, vp,
                                  vp, vp, sz, vp]
    lib.gnca_step_phases_f32.restype = ctypes.c_int
    lib.gnca_step_phases_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights), vp, vp,
                                         vp, vp, vp, sz, vp, ctypes.c_uint32]
    lib.gnca_message_f32.restype = ctypes.c_int
    lib.gnca_message_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights), vp, vp,
                                     vp, vp, sz, vp]
    lib.gnca_perceive_f32.restype = ctypes.c_int
    lib.gnca_perceive_f32.argtypes = [ctypes.c_int32] * 4 + [vp, vp, vp, vp]
    lib.gnca_rollout_f32.restype = ctypes.c_int
    lib.gnca_rollout_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights),
                                     ctypes.c_int32, vp, vp, vp, vp, vp, sz, vp]
    lib.gnca_rollout_ex_f32.restype = ctypes.c_int
    lib.gnca_rollout_ex_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights),
                                        ctypes.c_int32, vp, vp, vp, vp, vp, sz, ctypes.c_uint32, vp]
    lib.gnca_rollout_stamped_f32.restype = ctypes.c_int
    lib.gnca_rollout_stamped_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights),
                                             ctypes.c_int32, vp, vp, vp, vp, vp, sz, vp,
                                             ctypes.c_int32, vp]
    lib.gnca_fire_mask_u8.restype = ctypes.c_int
    lib.gnca_fire_mask_u8.argtypes = [ctypes.POINTER(StepDesc), vp, vp]
    lib.gnca_bwd_workspace_bytes.restype = sz
    lib.gnca_bwd_workspace_bytes.argtypes = [ctypes.POINTER(StepDesc)]
    lib.gnca_step_bwd_f32.restype = ctypes.c_int
    lib.gnca_step_bwd_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights), vp, vp, vp,
                                      vp, vp, ctypes.POINTER(Grads), vp, vp, sz, vp]
    i32, i64 = ctypes.c_int32, ctypes.c_int64
    lib.gnca_loss_premult_f32.restype = ctypes.c_int
    lib.gnca_loss_premult_f32.argtypes = [i32, i32, i32, vp, i64, vp, i64, vp, vp]
    lib.gnca_loss_premult_bwd_f32.restype = ctypes.c_int
    lib.gnca_loss_premult_bwd_f32.argtypes = [i32, i32, i32, vp, i64, vp, i64, vp, vp, i64, vp]
    lib.gnca_damage_f32.restype = ctypes.c_int
    lib.gnca_damage_f32.argtypes = [ctypes.POINTER(DamageDesc), vp, vp, vp, vp]
    lib.gnca_k1_variant.restype = ctypes.c_int
    lib.gnca_k1_variant.argtypes = [ctypes.POINTER(StepDesc), ctypes.c_char_p, i32, ctypes.POINTER(ctypes.c_int32)]
    lib.gnca_bb_variant.restype = ctypes.c_int
    lib.gnca_bb_variant.argtypes = [ctypes.POINTER(StepDesc), ctypes.c_char_p, i32]
    lib.gnca_step_masked_f32.restype = ctypes.c_int
    lib.gnca_step_masked_f32.argtypes = [ctypes.POINTER(StepDesc), ctypes.POINTER(Weights), vp, vp, vp,
                                         vp, vp, sz, vp]
    v = lib.gnca_abi_version()
    if v != ABI_VERSION:
        raise GncaError(f"libgnca.so ABI version {v} != expected {ABI_VERSION}; rebuild it")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        lib = load()
        msg = lib.gnca_status_string(rc).decode()
        hip = lib.gnca_last_hip_error()
        raise GncaError(f"{what} failed: {msg} (status {rc}, hipError {hip})")
