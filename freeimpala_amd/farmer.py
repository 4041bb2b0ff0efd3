"""Host side of the MI355X FarmerLstm train step (include/fi_farmer.h), shaped like the
reference's own Python interface (/root/reference/scripts/gpu_benchmark.py):

  FarmerLstmModel            the model (gpu_benchmark.py:11-44); its parameters live on the
                             device as one fp32 blob in state_dict order
  get_loss_function(name)    'mse' / 'mae' / 'huber' (gpu_benchmark.py:46-55; same errors)
  get_optimizer(type, model, lr)  'adam' / 'sgd' / 'adamw' (gpu_benchmark.py:57-66)
  generate_synthetic_data    z [B,T,162], x [B,484], targets [B,1] (gpu_benchmark.py:86-97)
  run_single_training_iteration(model, z, x, targets, criterion, optimizer, device)
                             -> (elapsed seconds, loss)   (gpu_benchmark.py:99-125)

Everything runs in HIP kernels of libfi_learner.so (farmer.hip); there is no CPU path: the
library missing or no device present raises. Arrays are numpy (host) -- copied in per step --
or the handle's resident device buffers (upload_inputs + train_step_resident)."""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _abi
from . import hip

I_IN, HID, X_IN = 162, 128, 484
LOSSES = {"mse": 0, "mae": 1, "huber": 2}
OPTIMIZERS = {"adam": 0, "sgd": 1, "adamw": 2}


class FarmerConfig(C.Structure):
    _fields_ = [("batch", C.c_int32), ("seq_len", C.c_int32), ("loss", C.c_int32),
                ("optimizer", C.c_int32), ("lr", C.c_float), ("beta1", C.c_float),
                ("beta2", C.c_float), ("eps", C.c_float), ("weight_decay", C.c_float),
                ("device", C.c_int32)]


class FarmerStats(C.Structure):
    _fields_ = [("loss", C.c_double), ("step_ms", C.c_float), ("step", C.c_uint64)]


_P = C.c_void_p
SIGNATURES = {  # every symbol include/fi_farmer.h declares
    "fi_farmer_param_count": ([], C.c_size_t),
    "fi_farmer_config_init": ([C.POINTER(FarmerConfig)], None),
    "fi_farmer_create": ([C.POINTER(FarmerConfig), C.POINTER(_P)], C.c_int),
    "fi_farmer_destroy": ([_P], None),
    "fi_farmer_set_params": ([_P, _P, C.c_size_t], C.c_int),
    "fi_farmer_get_params": ([_P, _P, C.c_size_t], C.c_int),
    "fi_farmer_get_grads": ([_P, _P, C.c_size_t], C.c_int),
    "fi_farmer_train_step": ([_P, _P, _P, _P, C.c_int, _P, C.POINTER(FarmerStats)], C.c_int),
    "fi_farmer_forward": ([_P, _P, _P, C.c_int, _P], C.c_int),
    "fi_farmer_tensor": ([_P, C.c_char_p, C.POINTER(_P), C.POINTER(C.c_size_t)], C.c_int),
    "fi_farmer_stream": ([_P], _P),
    "fi_farmer_set_profiling": ([_P, C.c_int], C.c_int),
    "fi_farmer_recurrence_ms": ([_P, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_int)], C.c_int),
}
_bound = None


def lib():
    global _bound
    L = _abi.lib()
    if _bound is not L:
        for name, (args, res) in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _bound = L
    return L


def param_count() -> int:
    return int(lib().fi_farmer_param_count())


class Criterion:
    def __init__(self, name: str):
        self.name = name.lower()
        self.kind = LOSSES[self.name]


def get_loss_function(loss_function_name: str) -> Criterion:
    if loss_function_name.lower() not in LOSSES:
        raise ValueError(f"Unsupported loss function: {loss_function_name}")
    return Criterion(loss_function_name)


class OptimizerSpec:
    def __init__(self, kind: str, lr: float, weight_decay: float | None = None):
        self.kind, self.lr, self.weight_decay = kind.lower(), float(lr), weight_decay


def get_optimizer(optimizer_type: str, model_parameters=None, learning_rate: float = 1e-3) -> OptimizerSpec:
    if optimizer_type.lower() not in OPTIMIZERS:
        raise ValueError(f"Unsupported optimizer: {optimizer_type}")
    return OptimizerSpec(optimizer_type, learning_rate)


def generate_synthetic_data(batch_size: int, seq_length: int, device=None, seed: int = 0):
    rs = np.random.RandomState(seed)
    z = rs.standard_normal((batch_size, seq_length, I_IN)).astype(np.float32)
    x = rs.standard_normal((batch_size, X_IN)).astype(np.float32)
    t = rs.standard_normal((batch_size, 1)).astype(np.float32)
    return z, x, t


class FarmerLstmModel:
    """The device-resident model + its train step. batch_size / seq_length are fixed per handle
    (the device buffers are sized for them); criterion and optimizer are chosen at creation
    (the reference builds them once per run too, gpu_benchmark.py:355-359)."""

    def __init__(self, batch_size: int = 32, seq_length: int = 10, loss: str = "mse",
                 optimizer: str = "adam", lr: float = 1e-3, weight_decay: float | None = None,
                 device: int = 0, params: np.ndarray | None = None):
        cfg = FarmerConfig()
        lib().fi_farmer_config_init(C.byref(cfg))
        cfg.batch, cfg.seq_len = batch_size, seq_length
        cfg.loss, cfg.optimizer = LOSSES[loss.lower()], OPTIMIZERS[optimizer.lower()]
        cfg.lr, cfg.device = lr, device
        if weight_decay is not None:
            cfg.weight_decay = weight_decay
        h = _P()
        _abi.check(lib().fi_farmer_create(C.byref(cfg), C.byref(h)), "fi_farmer_create")
        self._h = h
        self.B, self.T = batch_size, seq_length
        self.loss_name, self.optimizer_name, self.lr = loss, optimizer, lr
        if params is not None:
            self.set_params(params)

    def close(self):
        if getattr(self, "_h", None):
            lib().fi_farmer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, p: np.ndarray) -> None:
        p = np.ascontiguousarray(p, np.float32)
        _abi.check(lib().fi_farmer_set_params(self._h, p.ctypes.data, p.size), "fi_farmer_set_params")

    def get_params(self) -> np.ndarray:
        out = np.empty(param_count(), np.float32)
        _abi.check(lib().fi_farmer_get_params(self._h, out.ctypes.data, out.size), "fi_farmer_get_params")
        return out

    def get_grads(self) -> np.ndarray:
        out = np.empty(param_count(), np.float32)
        _abi.check(lib().fi_farmer_get_grads(self._h, out.ctypes.data, out.size), "fi_farmer_get_grads")
        return out

    def tensor(self, name: str):
        p, n = _P(), C.c_size_t()
        _abi.check(lib().fi_farmer_tensor(self._h, name.encode(), C.byref(p), C.byref(n)), "fi_farmer_tensor")
        return p.value, n.value

    def tensor_array(self, name: str, shape, dtype=np.float32) -> np.ndarray:
        """A copy of a named device tensor (fi_farmer_tensor) as a host array, after the
        handle's stream has finished."""
        p, n = self.tensor(name)
        hip.synchronize()
        a = hip.download_ptr(p, dtype, (n // np.dtype(dtype).itemsize,))
        return a.reshape(shape)

    def _check_shapes(self, z, x, t=None):
        assert z.shape == (self.B, self.T, I_IN) and x.shape == (self.B, X_IN), (z.shape, x.shape)
        if t is not None:
            assert t.size == self.B, t.shape

    def train_step(self, z, x, targets, with_values=False):
        """One reference train step on host arrays: returns the loss (and the forward values)."""
        z, x, t = (np.ascontiguousarray(a, np.float32) for a in (z, x, targets))
        self._check_shapes(z, x, t)
        st = FarmerStats()
        vals = np.empty(self.B, np.float32) if with_values else None
        _abi.check(lib().fi_farmer_train_step(self._h, z.ctypes.data, x.ctypes.data, t.ctypes.data, 0,
                                              vals.ctypes.data if vals is not None else None, C.byref(st)),
                   "fi_farmer_train_step")
        self.last_step_ms = st.step_ms
        return (st.loss, vals.reshape(self.B, 1)) if with_values else st.loss

    def train_step_resident(self, stats: bool = True):
        """One step on the handle's own device input buffers (z / x / targets already in HBM)."""
        zp, xp, tp = (self.tensor(n)[0] for n in ("z", "x", "targets"))
        st = FarmerStats()
        _abi.check(lib().fi_farmer_train_step(self._h, zp, xp, tp, 1, None, C.byref(st) if stats else None),
                   "fi_farmer_train_step")
        if stats:
            self.last_step_ms = st.step_ms
        return st.loss if stats else None

    def recurrence_ms(self, steps: int = 5):
        """Mean device ms of the two recurrence kernels (forward LSTM, BPTT) over `steps`
        resident train steps, from HIP events around each launch (bench roofline)."""
        _abi.check(lib().fi_farmer_set_profiling(self._h, 1), "fi_farmer_set_profiling")
        for _ in range(steps):
            self.train_step_resident(stats=False)
        f, b, n = C.c_float(), C.c_float(), C.c_int()
        _abi.check(lib().fi_farmer_recurrence_ms(self._h, C.byref(f), C.byref(b), C.byref(n)), "fi_farmer_recurrence_ms")
        _abi.check(lib().fi_farmer_set_profiling(self._h, 0), "fi_farmer_set_profiling")
        return f.value, b.value

    def upload_inputs(self, z, x, targets) -> None:
        for name, a in (("z", z), ("x", x), ("targets", targets)):
            p, n = self.tensor(name)
            a = np.ascontiguousarray(a, np.float32)
            assert a.nbytes == n, (name, a.nbytes, n)
            hip.upload_ptr(p, a)

    def __call__(self, z, x, return_value=True):
        """FarmerLstmModel.forward(z, x, return_value=True) -> {'values': [B, 1]}."""
        z, x = (np.ascontiguousarray(a, np.float32) for a in (z, x))
        self._check_shapes(z, x)
        vals = np.empty(self.B, np.float32)
        _abi.check(lib().fi_farmer_forward(self._h, z.ctypes.data, x.ctypes.data, 0, vals.ctypes.data),
                   "fi_farmer_forward")
        return dict(values=vals.reshape(self.B, 1))

    def sync(self):
        hip.synchronize()


def run_single_training_iteration(model: FarmerLstmModel, z, x, targets, criterion=None, optimizer=None,
                                  device=None):
    """gpu_benchmark.py:99-125: (elapsed seconds, loss). The criterion / optimizer are the
    model's (fixed at creation); passing others is an error rather than a silent mismatch."""
    if criterion is not None and criterion.name != model.loss_name.lower():
        raise ValueError(f"model was built with loss {model.loss_name}, not {criterion.name}")
    if optimizer is not None and optimizer.kind != model.optimizer_name.lower():
        raise ValueError(f"model was built with optimizer {model.optimizer_name}, not {optimizer.kind}")
    t0 = time.time()
    loss = model.train_step(z, x, targets)
    return time.time() - t0, loss
