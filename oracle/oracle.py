"""ctypes front-end of the CPU oracle (oracle/impala_oracle.c) -- TEST INFRASTRUCTURE.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import
this module; it is the checker, never the thing measured as the product. The product
(``freeimpala_amd``) never imports it (tests/test_no_oracle_in_product.py checks that).

The restated algorithm and its citations live in the C file header: reference
``include/freeimpala/learner.h:32-49`` (the step being replaced) and the IMPALA spec as
restated in SURVEY.md 8(a).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


class Hparams(C.Structure):
    _fields_ = [("rho_bar", C.c_double), ("c_bar", C.c_double), ("pg_rho_bar", C.c_double),
                ("lambda_", C.c_double), ("baseline_cost", C.c_double),
                ("entropy_cost", C.c_double)]


DEFAULT_HP = dict(rho_bar=1.0, c_bar=1.0, pg_rho_bar=1.0, lambda_=1.0,
                  baseline_cost=0.5, entropy_cost=0.01)


def build() -> str:
    """Compile the oracle with its Makefile (gcc). Returns the .so path."""
    src = os.path.join(_HERE, "impala_oracle.c")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.orc_vtrace_loss.argtypes = [C.c_int, C.c_int, C.c_int, P, P, P, P, P, P,
                                      C.POINTER(Hparams), P, P, P, P, P]
        L.orc_vtrace_loss.restype = C.c_int
        L.orc_mlp_param_count.argtypes = [C.c_int, C.c_int, C.c_int]
        L.orc_mlp_param_count.restype = C.c_size_t
        L.orc_mlp_forward.argtypes = [C.c_int] * 4 + [P] * 5
        L.orc_mlp_backward.argtypes = [C.c_int] * 4 + [P] * 6
        L.orc_atari_param_count.argtypes = [C.c_int]
        L.orc_atari_param_count.restype = C.c_size_t
        L.orc_atari_forward.argtypes = [C.c_int, C.c_int, P, P, C.c_int, P, P, P, P, P]
        L.orc_atari_backward.argtypes = [C.c_int, C.c_int, P, P, C.c_int, P, P, P, P, P, P]
        L.orc_atari_backward_ex.argtypes = [C.c_int, C.c_int, P, P, C.c_int] + [P] * 10
        L.orc_clip_grad_norm.argtypes = [C.c_size_t, P, C.c_double]
        L.orc_clip_grad_norm.restype = C.c_double
        L.orc_adam.argtypes = [C.c_size_t, P, P, P, P, C.c_float, C.c_float, C.c_float,
                               C.c_float, C.c_int]
        L.orc_sgd.argtypes = [C.c_size_t, P, P, C.c_float]
        L.orc_philox4.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, P]
        L.orc_synth_batch.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, C.c_float, P, P, P, P, P, P]
        L.orc_conv_wgrad_f64.argtypes = [C.c_int] * 6 + [P, C.c_int, P, C.c_int, P, P]
        L.orc_conv_wgrad_f64.restype = C.c_int
        L.orc_bf16_round.argtypes = [C.c_float]
        L.orc_bf16_round.restype = C.c_float
        L.orc_num_threads.restype = C.c_int
        L.orc_set_num_threads.argtypes = [C.c_int]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def vtrace_loss(pi, mu, actions, rewards, discounts, values, **hp):
    """pi, mu: (T,B,A) f32; actions (T,B) i32; rewards/discounts (T,B); values (T+1,B).
    Returns dict(vs, pg_adv, dlogits, dvalue, losses[pg, baseline, entropy])."""
    pi, mu = _f32(pi), _f32(mu)
    T, B, A = pi.shape
    actions = np.ascontiguousarray(actions, dtype=np.int32)
    rewards, discounts, values = _f32(rewards), _f32(discounts), _f32(values)
    assert mu.shape == (T, B, A) and actions.shape == (T, B) and values.shape == (T + 1, B)
    h = dict(DEFAULT_HP)
    h.update(hp)
    H = Hparams(**h)
    vs = np.empty((T, B), np.float32)
    adv = np.empty((T, B), np.float32)
    dl = np.empty((T, B, A), np.float32)
    dv = np.empty((T + 1, B), np.float32)
    losses = np.zeros(3, np.float64)
    rc = lib().orc_vtrace_loss(T, B, A, _p(pi), _p(mu), _p(actions), _p(rewards),
                               _p(discounts), _p(values), C.byref(H), _p(vs), _p(adv),
                               _p(dl), _p(dv), _p(losses))
    if rc != 0:
        raise ValueError(f"orc_vtrace_loss failed rc={rc}")
    return dict(vs=vs, pg_adv=adv, dlogits=dl, dvalue=dv, losses=losses)


def total_loss(losses, baseline_cost=0.5, entropy_cost=0.01):
    return float(losses[0] + baseline_cost * losses[1] + entropy_cost * losses[2])


def mlp_param_count(D=128, H=256, A=18):
    return int(lib().orc_mlp_param_count(D, H, A))


def mlp_forward(obs, params, H=256, A=18):
    obs = _f32(obs)
    N, D = obs.shape
    params = _f32(params)
    h1 = np.empty((N, H), np.float32)
    h2 = np.empty((N, H), np.float32)
    out = np.empty((N, A + 1), np.float32)
    rc = lib().orc_mlp_forward(N, D, H, A, _p(obs), _p(params), _p(h1), _p(h2), _p(out))
    assert rc == 0
    return h1, h2, out


def mlp_backward(obs, params, h1, h2, dout, H=256, A=18):
    obs = _f32(obs)
    N, D = obs.shape
    g = np.empty(mlp_param_count(D, H, A), np.float32)
    rc = lib().orc_mlp_backward(N, D, H, A, _p(obs), _p(_f32(params)), _p(_f32(h1)),
                                _p(_f32(h2)), _p(_f32(dout)), _p(g))
    assert rc == 0
    return g


def atari_param_count(A=18):
    return int(lib().orc_atari_param_count(A))


def atari_forward(frames, params, A=18, bf16_emul=True):
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    N = frames.shape[0]
    a1 = np.empty((N, 20, 20, 32), np.float32)
    a2 = np.empty((N, 9, 9, 64), np.float32)
    a3 = np.empty((N, 7, 7, 64), np.float32)
    h = np.empty((N, 512), np.float32)
    out = np.empty((N, A + 1), np.float32)
    rc = lib().orc_atari_forward(N, A, _p(frames), _p(_f32(params)), int(bf16_emul), _p(a1),
                                 _p(a2), _p(a3), _p(h), _p(out))
    assert rc == 0
    return dict(a1=a1, a2=a2, a3=a3, h=h, out=out)


def atari_backward(frames, params, acts, dout, A=18, bf16_emul=True):
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    N = frames.shape[0]
    g = np.empty(atari_param_count(A), np.float32)
    rc = lib().orc_atari_backward(N, A, _p(frames), _p(_f32(params)), int(bf16_emul),
                                  _p(acts["a1"]), _p(acts["a2"]), _p(acts["a3"]),
                                  _p(acts["h"]), _p(_f32(dout)), _p(g))
    assert rc == 0
    return g


def atari_backward_ex(frames, params, acts, dout, A=18, bf16_emul=True):
    """Returns (grads, dict(dh, d3, d2, d1)) -- the masked data gradients of every layer."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    N = frames.shape[0]
    g = np.empty(atari_param_count(A), np.float32)
    mids = dict(dh=np.empty((N, 512), np.float32), d3=np.empty((N, 7, 7, 64), np.float32),
                d2=np.empty((N, 9, 9, 64), np.float32), d1=np.empty((N, 20, 20, 32), np.float32))
    rc = lib().orc_atari_backward_ex(N, A, _p(frames), _p(_f32(params)), int(bf16_emul),
                                     _p(acts["a1"]), _p(acts["a2"]), _p(acts["a3"]), _p(acts["h"]),
                                     _p(_f32(dout)), _p(g), _p(mids["dh"]), _p(mids["d3"]),
                                     _p(mids["d2"]), _p(mids["d1"]))
    assert rc == 0
    return g, mids


def clip_grad_norm(g, max_norm):
    return float(lib().orc_clip_grad_norm(g.size, _p(g), max_norm))


def adam(p, g, m, v, lr, b1, b2, eps, step):
    lib().orc_adam(p.size, _p(p), _p(g), _p(m), _p(v), lr, b1, b2, eps, step)


def sgd(p, g, lr):
    lib().orc_sgd(p.size, _p(p), _p(g), lr)


def philox4(seed, e, stream):
    out = np.zeros(4, np.uint32)
    lib().orc_philox4(seed, e, stream, _p(out))
    return out


def synth_batch(seed, T, B, A=18, D=128, B_glob=None, b_off=0, gamma=0.99,
                obs=True, frames=False):
    B_glob = B if B_glob is None else B_glob
    o = np.empty((T + 1, B, D), np.float32) if obs else None
    fr = np.empty((T + 1, B, 84, 84, 4), np.uint8) if frames else None
    mu = np.empty((T, B, A), np.float32)
    act = np.empty((T, B), np.int32)
    rew = np.empty((T, B), np.float32)
    disc = np.empty((T, B), np.float32)
    lib().orc_synth_batch(seed, T, B, B_glob, b_off, A, D, gamma, _p(o), _p(mu), _p(act),
                          _p(rew), _p(disc), _p(fr))
    return dict(obs=o, frames=fr, mu=mu, actions=act, rewards=rew, discounts=disc)


def conv_wgrad_f64(X, dY, N, IH, IC, K, S, OC, cos, x_kind):
    """fp64 weight gradient of a strided VALID conv for output channels `cos` from stored operands
    (X: uint8 frames (x_kind 0), bf16 bits NHWC (1) or in the parity-plane order (2); dY: bf16
    bits NHWC) -> (K, K, IC, len(cos)), unscaled. Checker for the full-depth gradient test."""
    X = np.ascontiguousarray(X)
    dY = np.ascontiguousarray(dY, np.uint16)
    assert X.dtype == (np.uint8 if x_kind == 0 else np.uint16) and X.size == N * IH * IH * IC
    OH = (IH - K) // S + 1
    assert dY.size == N * OH * OH * OC
    c = np.ascontiguousarray(cos, np.int32)
    out = np.zeros((K, K, IC, c.size), np.float64)
    rc = lib().orc_conv_wgrad_f64(N, IH, IC, K, S, OC, _p(X), x_kind, _p(dY), c.size, _p(c), _p(out))
    assert rc == 0, rc
    return out


def bf16_round(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    special = (x.view(np.uint32) & 0x7F800000) == 0x7F800000
    r = np.where(special, x.view(np.uint32), r)
    return r.view(np.float32)


def set_threads(n):
    lib().orc_set_num_threads(int(n))


def num_threads():
    return int(lib().orc_num_threads())
