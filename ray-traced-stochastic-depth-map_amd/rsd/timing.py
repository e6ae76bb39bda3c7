"""Timing-only HIP events (measurement plumbing for bench.py and tools/).

torch.cuda.Event records with the default flags, i.e. with a system-scope release fence: every
record writes back and invalidates the caches, which on MI355X leaves a ~5-6 us bubble in the
stream it is recorded in (the rocprof timeline of bench.py showed 5.8 us between pass 1 and the SD
trace exactly where an event sits, and none between the trace's two kernels).  Events created with
hipEventDisableSystemFence time the same stream order without that fence ("This can be used for
events that are only being used to measure timing", hip_runtime_api.h) -- they are what the bench's
per-kernel timings use.  The events come from the HIP runtime torch itself loaded (one runtime per
process), found in /proc/self/maps."""
from __future__ import annotations

import ctypes as C

_HIP = None
HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000


def _hip():
    global _HIP
    if _HIP is None:
        import torch
        torch.cuda.init()
        path = None
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64.so" in line:
                    path = line.split()[-1]
                    break
        if path is None:
            raise RuntimeError("libamdhip64 is not loaded in this process")
        L = C.CDLL(path)
        L.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
        L.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        L.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        L.hipEventDestroy.argtypes = [C.c_void_p]
        L.hipEventQuery.argtypes = [C.c_void_p]
        _HIP = L
    return _HIP


class TimingEvent:
    """A HIP event for timing only: record() on torch's current stream (or `stream`), elapsed_time()
    in milliseconds like torch.cuda.Event."""

    def __init__(self):
        self._L = _hip()
        self.h = C.c_void_p()
        if self._L.hipEventCreateWithFlags(C.byref(self.h), HIP_EVENT_DISABLE_SYSTEM_FENCE) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")

    def record(self, stream=None):
        import torch
        if stream is not None:
            s = stream.cuda_stream
        else:  # torch's raw accessor: no Python Stream object per record (3 us each through current_stream())
            s = torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
        if self._L.hipEventRecord(self.h, C.c_void_p(s)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def synchronize(self):
        """Block the host until the event has completed (hipEventSynchronize)."""
        if self._L.hipEventSynchronize(self.h) != 0:
            raise RuntimeError("hipEventSynchronize failed")

    def query(self) -> bool:
        """True when the event has completed (hipEventQuery; never blocks)."""
        return self._L.hipEventQuery(self.h) == 0

    def elapsed_time(self, end: "TimingEvent") -> float:
        ms = C.c_float()
        if self._L.hipEventElapsedTime(C.byref(ms), self.h, end.h) != 0:
            raise RuntimeError("hipEventElapsedTime failed (events not complete?)")
        return ms.value

    def __del__(self):
        try:
            if self.h:
                self._L.hipEventDestroy(self.h)
        except Exception:
            pass
