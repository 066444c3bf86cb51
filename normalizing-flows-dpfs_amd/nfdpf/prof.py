"""Live kernel timing with raw hipEvents (recorded by libnfdpf around the dominant launch
of a step, on the launch's own stream; see nfdpf_filter_desc.prof_events)."""
from __future__ import annotations

import ctypes
import os

import torch

_hip = None


def hip():
    global _hip
    if _hip is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        _hip = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        _hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        _hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        _hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        _hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        _hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return _hip


class EventPair:
    """hipEvents in a C array (the ABI's prof_events): one pair, or two with ``n=4`` (the
    tiled step's proposal launch, then its front launch -- nfdpf_filter_desc.prof_front)."""

    def __init__(self, n: int = 2):
        self.n = n
        self.arr = (ctypes.c_void_p * n)()
        for k in range(n):
            e = ctypes.c_void_p()
            rc = hip().hipEventCreate(ctypes.byref(e))
            if rc != 0:
                raise RuntimeError(f"hipEventCreate failed ({rc})")
            self.arr[k] = e.value

    @property
    def ptr(self) -> int:
        return ctypes.addressof(self.arr)

    def _record(self, k: int, device):
        from ._lib import stream_ptr
        rc = hip().hipEventRecord(self.arr[k], ctypes.c_void_p(stream_ptr(device)))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed ({rc})")

    def record_start(self, device):
        """Record event 0 on the stream the next nfdpf launch on ``device`` goes to."""
        self._record(0, device)

    def record_end(self, device):
        self._record(1, device)

    def ms(self, pair: int = 0) -> float:
        a, b = self.arr[2 * pair], self.arr[2 * pair + 1]
        hip().hipEventSynchronize(b)
        out = ctypes.c_float()
        rc = hip().hipEventElapsedTime(ctypes.byref(out), a, b)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed ({rc})")
        return float(out.value)

    def close(self):
        for k in range(self.n):
            if self.arr[k]:
                hip().hipEventDestroy(self.arr[k])
                self.arr[k] = None
