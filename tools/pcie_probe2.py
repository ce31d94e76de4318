#!/usr/bin/env python3
"""H2D / D2H rate from host memory page-locked three ways (hipHostMalloc,
hipHostRegister of numpy buffers, and registered buffers copied in 32-page
chunks on 8 streams, as the host-fed runner does), both directions at once.
ctypes on libamdhip64; tuning only."""
import ctypes as C
import time

import numpy as np

hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
hip.hipDeviceSynchronize.argtypes = []
H2D, D2H = 1, 2
PAGE = 2480 * 3508


def dmalloc(n):
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), n) == 0
    return p.value


def streams(k):
    out = []
    for _ in range(k):
        s = C.c_void_p()
        assert hip.hipStreamCreateWithFlags(C.byref(s), 1) == 0
        out.append(s.value)
    return out


def run(hin, hout, n, chunk, nst, reps=3):
    din, dout = dmalloc(n), dmalloc(n)
    st = streams(nst)
    def once():
        for i, off in enumerate(range(0, n, chunk)):
            m = min(chunk, n - off)
            s = st[i % nst]
            hip.hipMemcpyAsync(din + off, hin + off, m, H2D, s)
            hip.hipMemcpyAsync(hout + off, dout + off, m, D2H, s)
        hip.hipDeviceSynchronize()
    once()
    t = time.perf_counter()
    for _ in range(reps):
        once()
    dt = (time.perf_counter() - t) / reps
    return 2 * n / dt / 1e9, n / PAGE / dt


if __name__ == "__main__":
    n = 320 * PAGE  # 2.8 GB each way
    ph, po = C.c_void_p(), C.c_void_p()
    assert hip.hipHostMalloc(C.byref(ph), n, 0) == 0 and hip.hipHostMalloc(C.byref(po), n, 0) == 0
    for chunk, nst in ((n, 1), (32 * PAGE, 8), (8 * PAGE, 8)):
        gb, pps = run(ph.value, po.value, n, chunk, nst)
        print(f"hipHostMalloc  chunk {chunk // PAGE:3d} pages x {nst} streams: {gb:6.1f} GB/s both ways = {pps:7.0f} pages/s")
    a = np.ones(n, np.uint8)
    b = np.ones(n, np.uint8)
    assert hip.hipHostRegister(a.ctypes.data, n, 0) == 0 and hip.hipHostRegister(b.ctypes.data, n, 0) == 0
    for chunk, nst in ((n, 1), (32 * PAGE, 8), (8 * PAGE, 8)):
        gb, pps = run(a.ctypes.data, b.ctypes.data, n, chunk, nst)
        print(f"hipHostRegister chunk {chunk // PAGE:3d} pages x {nst} streams: {gb:6.1f} GB/s both ways = {pps:7.0f} pages/s")
