"""ctypes binding of libfi_learner.so (the C ABI declared in include/fi_learner.h).

This is the same binding a Python host of freeimpala would add (INTEGRATION.md shows it);
tests/, bench.py and smoke() drive the HIP learner through it. There is NO fallback: if
the in-tree HIP library is missing or fails to load, importing raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FI_LIB_OVERRIDE") or os.path.join(_HERE, "lib", "libfi_learner.so")  # override: A/B experiment builds only

FI_OK = 0
FI_ARCH_MLP, FI_ARCH_ATARI = 0, 1
FI_OPT_ADAM, FI_OPT_SGD = 0, 1
FI_PUBLISH_FP32, FI_PUBLISH_BF16 = 0, 1
PHASES = ["ingest", "forward", "vtrace", "backward", "allreduce", "optimizer"]
RECORD_BYTES = 1024
# record schema inside one 1 KiB ELEMENT
REC_OBS, REC_MU, REC_ACT, REC_REW, REC_DISC, REC_FLAGS = 0, 512, 768, 772, 776, 780


class VtraceHparams(C.Structure):
    _fields_ = [("rho_bar", C.c_float), ("c_bar", C.c_float), ("pg_rho_bar", C.c_float),
                ("lambda_", C.c_float), ("baseline_cost", C.c_float),
                ("entropy_cost", C.c_float)]


class LearnerConfig(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("arch", C.c_int32), ("seq_len", C.c_int32),
                ("batch", C.c_int32), ("num_actions", C.c_int32), ("obs_dim", C.c_int32),
                ("hidden", C.c_int32), ("optimizer", C.c_int32), ("publish_dtype", C.c_int32),
                ("device", C.c_int32), ("gamma", C.c_float), ("hp", VtraceHparams),
                ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float),
                ("eps", C.c_float), ("max_grad_norm", C.c_float), ("seed", C.c_uint64)]


class StepStats(C.Structure):
    _fields_ = [("pg_loss", C.c_double), ("baseline_loss", C.c_double),
                ("entropy_loss", C.c_double), ("total_loss", C.c_double),
                ("grad_norm", C.c_double), ("version", C.c_uint64), ("step_ms", C.c_float)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every symbol include/fi_learner.h declares, with its ctypes signature
_P = C.c_void_p
SIGNATURES = {
    "fi_abi_version": ([], C.c_int),
    "fi_last_error": ([], C.c_char_p),
    "fi_learner_config_init": ([C.POINTER(LearnerConfig)], None),
    "fi_learner_create": ([C.POINTER(LearnerConfig), C.POINTER(_P)], C.c_int),
    "fi_learner_destroy": ([_P], None),
    "fi_learner_param_count": ([_P], C.c_size_t),
    "fi_learner_param_bytes": ([_P], C.c_size_t),
    "fi_learner_entry_bytes": ([_P], C.c_size_t),
    "fi_learner_step": ([_P, C.POINTER(_P), C.c_size_t, C.c_size_t, C.POINTER(StepStats)], C.c_int),
    "fi_learner_step_async": ([_P, C.POINTER(_P), C.c_size_t, C.c_size_t], C.c_int),
    "fi_learner_wait": ([_P, C.POINTER(StepStats)], C.c_int),
    "fi_learner_acquire_staging": ([_P, C.POINTER(_P), C.POINTER(C.c_size_t)], C.c_int),
    "fi_learner_step_staged": ([_P, C.POINTER(StepStats)], C.c_int),
    "fi_learner_step_staged_async": ([_P], C.c_int),
    "fi_learner_state_bytes": ([_P], C.c_size_t),
    "fi_learner_save_state": ([_P, _P, C.c_size_t], C.c_int),
    "fi_learner_load_state": ([_P, _P, C.c_size_t], C.c_int),
    "fi_learner_step_resident": ([_P, C.POINTER(StepStats)], C.c_int),
    "fi_learner_synth_batch": ([_P, C.c_uint64, C.c_int32, C.c_int32], C.c_int),
    "fi_learner_get_params": ([_P, _P, C.c_size_t, C.POINTER(C.c_uint64)], C.c_int),
    "fi_learner_get_params_fp32": ([_P, _P, C.c_size_t], C.c_int),
    "fi_learner_set_params": ([_P, _P, C.c_size_t, C.c_uint64], C.c_int),
    "fi_comm_unique_id_bytes": ([], C.c_int),
    "fi_comm_get_unique_id": ([_P, C.c_size_t], C.c_int),
    "fi_learner_attach_comm": ([_P, _P, C.c_size_t, C.c_int, C.c_int], C.c_int),
    "fi_comm_init_all": ([_P, C.c_int], C.c_int),
    "fi_learner_comm_info": ([_P, _P, _P, _P], C.c_int),
    "fi_learner_tensor": ([_P, C.c_char_p, C.POINTER(_P), C.POINTER(C.c_size_t)], C.c_int),
    "fi_learner_read_tensor": ([_P, C.c_char_p, _P, C.c_size_t], C.c_int),
    "fi_learner_set_profiling": ([_P, C.c_int], C.c_int),
    "fi_learner_phase_times": ([_P, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)], C.c_int),
    "fi_learner_kernel_times": ([_P, C.c_char_p, C.c_size_t, C.POINTER(C.c_float),
                                 C.POINTER(C.c_int), C.c_int], C.c_int),
    "fi_learner_stream": ([_P], _P),
    "fi_learner_sync": ([_P], C.c_int),
    "fi_vtrace_workspace_bytes": ([C.c_int, C.c_int, C.c_int], C.c_size_t),
    "fi_vtrace_loss_fp32": ([C.c_int, C.c_int, C.c_int] + [_P] * 6 +
                            [C.POINTER(VtraceHparams)] + [_P] * 6 + [C.c_size_t, _P], C.c_int),
    "fi_vtrace_loss_fp32_variant": ([C.c_int, C.c_int, C.c_int, C.c_int] + [_P] * 6 +
                                    [C.POINTER(VtraceHparams)] + [_P] * 6 + [C.c_size_t, _P],
                                    C.c_int),
    "fi_ingest_records": ([_P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_size_t] + [_P] * 6,
                          C.c_int),
    "fi_synth_trajectories": ([C.c_uint64] + [C.c_int] * 6 + [C.c_float] + [_P] * 7, C.c_int),
}

_lib = None


class FiError(RuntimeError):
    pass


def lib():
    """Load the in-tree HIP library (raises if it is missing -- no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FiError(f"{LIB_PATH} not built: run `make` or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != FI_OK:
        msg = lib().fi_last_error().decode(errors="replace")
        raise FiError(f"{what} failed rc={rc}: {msg}")


def default_config(**kw) -> LearnerConfig:
    cfg = LearnerConfig()
    lib().fi_learner_config_init(C.byref(cfg))
    for k, v in kw.items():
        if k in ("rho_bar", "c_bar", "pg_rho_bar", "lambda_", "baseline_cost", "entropy_cost"):
            setattr(cfg.hp, k, v)
        else:
            setattr(cfg, k, v)
    return cfg
