"""Python handle over the HIP learner (C ABI ``fi_learner_*``).

Mirrors the surface freeimpala's C++ ``Learner`` exposes for the hot path
(reference include/freeimpala/learner.h): ``step(player_batch)`` is the body of
``Learner::trainModel(player_index, batch)`` (learner.h:32-49) where ``batch`` is what
``SharedBuffer::readBatch(M)`` returns (data_structures.h:267-300): M entries of
``entry_size * 1024`` bytes. The C++ Learner in include/freeimpala/learner.h calls the same
ABI; this module is the binding tests and bench.py use.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _abi
from ._abi import check, lib
from . import hip


class HostBatch:
    """M host entries pinned down once as a C pointer table (what Learner::step hands the ABI:
    `const void* const* entries`). Building the table costs ~1 us per entry in Python, so a
    caller that steps the same buffers repeatedly builds it once."""

    def __init__(self, batch: Sequence[bytes | bytearray | np.ndarray]):
        self.bufs = [np.frombuffer(e, dtype=np.uint8) if not isinstance(e, np.ndarray)
                     else np.ascontiguousarray(e).view(np.uint8).ravel() for e in batch]
        self.n = len(self.bufs)
        self.entry_bytes = min(b.nbytes for b in self.bufs) if self.bufs else 0
        self.ptrs = (C.c_void_p * self.n)(*[b.ctypes.data for b in self.bufs])


def _as_host_batch(batch) -> HostBatch:
    return batch if isinstance(batch, HostBatch) else HostBatch(batch)


class DeviceLearner:
    def __init__(self, arch: str = "mlp", seq_len: int = 100, batch: int = 32,
                 num_actions: int = 18, obs_dim: int = 128, hidden: int = 256,
                 optimizer: str = "adam", publish: str = "fp32", device: int = 0, **kw):
        self.cfg = _abi.default_config(
            arch=_abi.FI_ARCH_MLP if arch == "mlp" else _abi.FI_ARCH_ATARI, seq_len=seq_len,
            batch=batch, num_actions=num_actions, obs_dim=obs_dim, hidden=hidden,
            optimizer=_abi.FI_OPT_ADAM if optimizer == "adam" else _abi.FI_OPT_SGD,
            publish_dtype=_abi.FI_PUBLISH_FP32 if publish == "fp32" else _abi.FI_PUBLISH_BF16,
            device=device, **kw)
        self._h = C.c_void_p()
        check(lib().fi_learner_create(C.byref(self.cfg), C.byref(self._h)), "fi_learner_create")
        self.T, self.B, self.A = seq_len, batch, num_actions
        self.D, self.H = obs_dim, hidden
        self.arch = arch

    # --- sizes
    @property
    def param_count(self) -> int:
        return int(lib().fi_learner_param_count(self._h))

    @property
    def param_bytes(self) -> int:
        return int(lib().fi_learner_param_bytes(self._h))

    @property
    def entry_bytes(self) -> int:
        return int(lib().fi_learner_entry_bytes(self._h))

    # --- the step
    def step(self, batch: Sequence[bytes | bytearray | np.ndarray] | HostBatch,
             stats: bool = True) -> dict:
        """Learner::step(player, batch): batch = M SharedBuffer entries (host bytes)."""
        hb = _as_host_batch(batch)
        st = _abi.StepStats()
        check(lib().fi_learner_step(self._h, hb.ptrs, hb.n, hb.entry_bytes,
                                    C.byref(st) if stats else None), "fi_learner_step")
        return st.as_dict() if stats else {}

    def step_async(self, batch: Sequence[bytes | bytearray | np.ndarray] | HostBatch) -> None:
        """Stage the entries (copied before return) and enqueue the step; see wait()."""
        hb = _as_host_batch(batch)
        check(lib().fi_learner_step_async(self._h, hb.ptrs, hb.n, hb.entry_bytes),
              "fi_learner_step_async")

    def acquire_staging(self) -> np.ndarray:
        """The next pinned staging buffer as a writable (B, entry_bytes) uint8 view
        (SharedBuffer::readBatchInto's destination); valid until it is submitted."""
        dst, stride = C.c_void_p(), C.c_size_t()
        check(lib().fi_learner_acquire_staging(self._h, C.byref(dst), C.byref(stride)),
              "fi_learner_acquire_staging")
        buf = (C.c_uint8 * (self.B * stride.value)).from_address(dst.value)
        return np.frombuffer(buf, np.uint8).reshape(self.B, stride.value)

    def step_staged(self, stats: bool = True) -> dict:
        st = _abi.StepStats()
        check(lib().fi_learner_step_staged(self._h, C.byref(st) if stats else None),
              "fi_learner_step_staged")
        return st.as_dict() if stats else {}

    def step_staged_async(self) -> None:
        check(lib().fi_learner_step_staged_async(self._h), "fi_learner_step_staged_async")

    def wait(self) -> dict:
        st = _abi.StepStats()
        check(lib().fi_learner_wait(self._h, C.byref(st)), "fi_learner_wait")
        return st.as_dict()

    def save_state(self) -> bytes:
        n = lib().fi_learner_state_bytes(self._h)
        buf = (C.c_char * n)()
        check(lib().fi_learner_save_state(self._h, buf, n), "fi_learner_save_state")
        return bytes(buf)

    def load_state(self, blob: bytes) -> None:
        check(lib().fi_learner_load_state(self._h, blob, len(blob)), "fi_learner_load_state")

    def step_resident(self, stats: bool = True) -> dict | None:
        st = _abi.StepStats()
        check(lib().fi_learner_step_resident(self._h, C.byref(st) if stats else None),
              "fi_learner_step_resident")
        return st.as_dict() if stats else None

    def synth(self, seed: int = 42, b_global: int = 0, b_offset: int = 0) -> None:
        check(lib().fi_learner_synth_batch(self._h, seed, b_global, b_offset), "synth")

    def sync(self) -> None:
        check(lib().fi_learner_sync(self._h), "sync")

    @property
    def stream(self) -> int:
        return lib().fi_learner_stream(self._h)

    # --- params
    def get_params(self) -> np.ndarray:
        out = np.empty(self.param_count, np.float32)
        check(lib().fi_learner_get_params_fp32(self._h, out.ctypes.data, out.size), "get_params")
        return out

    def get_blob(self) -> tuple[bytes, int]:
        buf = (C.c_char * self.param_bytes)()
        ver = C.c_uint64(0)
        check(lib().fi_learner_get_params(self._h, buf, self.param_bytes, C.byref(ver)),
              "get_params")
        return bytes(buf), ver.value

    def set_params(self, p: np.ndarray | bytes, version: int = 0) -> None:
        a = np.frombuffer(p, np.uint8) if isinstance(p, (bytes, bytearray)) else np.ascontiguousarray(p)
        check(lib().fi_learner_set_params(self._h, a.ctypes.data, a.nbytes, version), "set_params")

    # --- tensors
    def tensor_ptr(self, name: str) -> tuple[int, int]:
        p = C.c_void_p()
        n = C.c_size_t()
        check(lib().fi_learner_tensor(self._h, name.encode(), C.byref(p), C.byref(n)), name)
        return p.value, n.value

    def tensor(self, name: str, dtype=np.float32, shape=None) -> np.ndarray:
        p, n = self.tensor_ptr(name)
        self.sync()
        a = hip.download_ptr(p, dtype, (n // np.dtype(dtype).itemsize,))
        return a.reshape(shape) if shape is not None else a

    def upload(self, name: str, a: np.ndarray) -> None:
        p, n = self.tensor_ptr(name)
        assert np.ascontiguousarray(a).nbytes == n, (name, a.nbytes, n)
        self.sync()
        hip.upload_ptr(p, a)

    def replay_vtrace(self, n: int = 20, sets: int = 1) -> float:
        """Mean device ms of the fused V-trace kernel alone: n back-to-back launches of
        fi_vtrace_loss_fp32 (no loss finalisation), HIP events around the burst.

        sets = 1: every launch reads this learner's resident tensors (~100 MB at T=100,
        B=4096), which stay in the 256 MB Infinity Cache between launches -- a WARM figure.
        sets = k > 1: launches rotate over k disjoint copies of the inputs and outputs
        (k x ~100 MB, > 256 MB for k >= 3), so each launch finds its tensors evicted by the
        k-1 launches before it -- the COLD (HBM) figure. Inputs are read-only and the
        learner's own outputs are rewritten with identical values: its state is unchanged."""
        T, B, A = self.T, self.B, self.A
        names = ("logits", "mu", "actions", "rewards", "discounts", "values", "vs", "pg_adv",
                 "dlogits", "dvalue")
        base = {k: self.tensor_ptr(k) for k in names}
        hp = self.cfg.hp
        wsb = lib().fi_vtrace_workspace_bytes(T, B, A)
        stream = self.stream
        self.sync()
        owned = []
        sets_ptr = [{k: v[0] for k, v in base.items()}]
        for _ in range(1, max(1, sets)):
            d = {}
            for k, (ptr, nb) in base.items():
                buf = hip.DeviceBuffer(nb)
                hip.copy_d2d(buf.ptr, ptr, nb)
                owned.append(buf)
                d[k] = buf.ptr
            sets_ptr.append(d)
        ws = [hip.DeviceBuffer(wsb) for _ in sets_ptr]

        def launch(i):
            ptr, w = sets_ptr[i % len(sets_ptr)], ws[i % len(sets_ptr)]
            check(lib().fi_vtrace_loss_fp32(
                T, B, A, ptr["logits"], ptr["mu"], ptr["actions"], ptr["rewards"], ptr["discounts"],
                ptr["values"], C.byref(hp), ptr["vs"], ptr["pg_adv"], ptr["dlogits"], ptr["dvalue"],
                None, w.ptr, wsb, stream), "fi_vtrace_loss_fp32")

        for i in range(max(3, len(sets_ptr))):
            launch(i)
        e0, e1 = hip.Event(), hip.Event()
        e0.record(stream)
        for i in range(n):
            launch(i)
        e1.record(stream)
        self.sync()
        ms = e0.elapsed_ms(e1) / n
        for b in owned + ws:
            b.free()
        return ms

    # --- data parallel
    @staticmethod
    def comm_unique_id() -> bytes:
        n = lib().fi_comm_unique_id_bytes()
        buf = (C.c_char * n)()
        check(lib().fi_comm_get_unique_id(buf, n), "comm_unique_id")
        return bytes(buf)

    def attach_comm(self, uid: bytes, rank: int, nranks: int) -> None:
        check(lib().fi_learner_attach_comm(self._h, uid, len(uid), rank, nranks), "attach_comm")

    def comm_info(self) -> dict:
        """RCCL's view of this handle's communicator and the gradient buckets of its last step."""
        n, r, b = C.c_int(), C.c_int(), C.c_int()
        check(lib().fi_learner_comm_info(self._h, C.byref(n), C.byref(r), C.byref(b)), "comm_info")
        return {"nranks": n.value, "rank": r.value, "buckets_last_step": b.value}

    @staticmethod
    def comm_init_all(learners) -> None:
        """One process, several devices: all handles join one communicator (rank = list index)."""
        arr = (C.c_void_p * len(learners))(*[x._h for x in learners])
        check(lib().fi_comm_init_all(arr, len(learners)), "comm_init_all")

    # --- profiling
    def set_profiling(self, on: bool) -> None:
        check(lib().fi_learner_set_profiling(self._h, int(on)), "set_profiling")

    def phase_times(self) -> dict:
        ms = (C.c_float * len(_abi.PHASES))()
        n = C.c_int(0)
        check(lib().fi_learner_phase_times(self._h, ms, len(_abi.PHASES), C.byref(n)), "phases")
        d = dict(zip(_abi.PHASES, list(ms)))
        d["steps"] = n.value
        return d

    def close(self) -> None:
        if self._h:
            lib().fi_learner_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_records(obs, mu, actions, rewards, discounts, entry_size=None) -> list[bytes]:
    """Build SharedBuffer entries from time-major arrays (inverse of the ingest kernel).
    obs (T+1,B,D), mu (T,B,A), actions/rewards/discounts (T,B). Returns B entries of
    entry_size*1024 bytes (default T+1 elements)."""
    T1, B, D = obs.shape
    T = T1 - 1
    A = mu.shape[-1]
    S = entry_size or T1
    out = []
    for b in range(B):
        e = np.zeros((S, 1024), np.uint8)
        rec = e[:T1]
        rec[:, 0:4 * D] = np.ascontiguousarray(obs[:, b, :], np.float32).view(np.uint8)
        rec[:T, 512:512 + 4 * A] = np.ascontiguousarray(mu[:, b, :], np.float32).view(np.uint8)
        rec[:T, 768:772] = np.ascontiguousarray(actions[:, b], np.int32).view(np.uint8).reshape(T, 4)
        rec[:T, 772:776] = np.ascontiguousarray(rewards[:, b], np.float32).view(np.uint8).reshape(T, 4)
        rec[:T, 776:780] = np.ascontiguousarray(discounts[:, b], np.float32).view(np.uint8).reshape(T, 4)
        out.append(e.tobytes())
    return out
