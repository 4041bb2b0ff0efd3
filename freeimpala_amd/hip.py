"""Minimal HIP runtime access over ctypes (device buffers, copies, sync, events).

Used by tests/bench to move numpy arrays in and out of HBM and to hand device pointers to
the C ABI. (torch is not needed for this; it is used only for torch.distributed.)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

_hip = None
H2D, D2H, D2D = 1, 2, 3


def hip():
    global _hip
    if _hip is None:
        # by soname: the runtime libfi_learner.so is bound to (the image's, or torch's copy
        # when torch was imported first), never a second HIP runtime in the process
        L = C.CDLL("libamdhip64.so.7")
        L.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        L.hipFree.argtypes = [C.c_void_p]
        L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        L.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        L.hipDeviceSynchronize.argtypes = []
        L.hipSetDevice.argtypes = [C.c_int]
        L.hipGetDeviceCount.argtypes = [C.POINTER(C.c_int)]
        L.hipGetErrorString.argtypes = [C.c_int]
        L.hipGetErrorString.restype = C.c_char_p
        L.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
        L.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        L.hipEventSynchronize.argtypes = [C.c_void_p]
        L.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        L.hipEventDestroy.argtypes = [C.c_void_p]
        L.hipStreamSynchronize.argtypes = [C.c_void_p]
        _hip = L
    return _hip


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {hip().hipGetErrorString(rc).decode()}")


def device_count() -> int:
    n = C.c_int(0)
    try:
        rc = hip().hipGetDeviceCount(C.byref(n))
    except OSError:
        return 0
    return n.value if rc == 0 else 0


def set_device(d: int) -> None:
    _chk(hip().hipSetDevice(d), "hipSetDevice")


def synchronize() -> None:
    _chk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceBuffer:
    """An owned hipMalloc allocation."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _chk(hip().hipMalloc(C.byref(p), max(16, self.nbytes)), "hipMalloc")
        self.ptr = p.value

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        _chk(hip().hipMemcpy(self.ptr, a.ctypes.data, a.nbytes, H2D), "hipMemcpy H2D")

    def download(self, dtype, shape) -> np.ndarray:
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        _chk(hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H), "hipMemcpy D2H")
        return out

    def zero(self) -> None:
        _chk(hip().hipMemset(self.ptr, 0, self.nbytes), "hipMemset")

    def free(self) -> None:
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def download_ptr(ptr: int, dtype, shape) -> np.ndarray:
    out = np.empty(shape, dtype)
    _chk(hip().hipMemcpy(out.ctypes.data, ptr, out.nbytes, D2H), "hipMemcpy D2H")
    return out


def copy_d2d(dst: int, src: int, nbytes: int) -> None:
    _chk(hip().hipMemcpy(dst, src, nbytes, D2D), "hipMemcpy D2D")


def upload_ptr(ptr: int, a: np.ndarray) -> None:
    a = np.ascontiguousarray(a)
    _chk(hip().hipMemcpy(ptr, a.ctypes.data, a.nbytes, H2D), "hipMemcpy H2D")


class Event:
    def __init__(self):
        e = C.c_void_p()
        _chk(hip().hipEventCreate(C.byref(e)), "hipEventCreate")
        self.e = e.value

    def record(self, stream=None):
        _chk(hip().hipEventRecord(self.e, stream), "hipEventRecord")

    def elapsed_ms(self, later: "Event") -> float:
        _chk(hip().hipEventSynchronize(later.e), "hipEventSynchronize")
        ms = C.c_float(0)
        _chk(hip().hipEventElapsedTime(C.byref(ms), self.e, later.e), "hipEventElapsedTime")
        return ms.value

    def __del__(self):
        try:
            hip().hipEventDestroy(self.e)
        except Exception:
            pass
