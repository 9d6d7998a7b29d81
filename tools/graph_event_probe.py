"""Can HIP event records be graph nodes (hipEventRecordExternal) inside a
torch stream capture on this ROCm?  Tries the capture modes and reports the
return codes and, if it works, the timed interval of a kernel in a replay."""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
hip.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
hip.hipGetLastError.restype = ctypes.c_int


def ev():
    e = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 0) == 0
    return e


x = torch.randn(4096, 4096, device="cuda")
for mode in ("global", "thread_local", "relaxed"):
    a, b = ev(), ev()
    g = torch.cuda.CUDAGraph()
    rcs = []
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            s = torch.cuda.current_stream().cuda_stream
            rcs.append(hip.hipEventRecordWithFlags(a, ctypes.c_void_p(s), 1))
            y = x @ x
            rcs.append(hip.hipEventRecordWithFlags(b, ctypes.c_void_p(s), 1))
        g.replay()
        torch.cuda.synchronize()
        ms = ctypes.c_float(0)
        rc = hip.hipEventElapsedTime(ctypes.byref(ms), a, b)
        print(mode, "record rcs", rcs, "elapsed rc", rc, "ms", ms.value, flush=True)
    except Exception as e:
        print(mode, "record rcs", rcs, "failed:", str(e).splitlines()[0], flush=True)
        hip.hipGetLastError()
