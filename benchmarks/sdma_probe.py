#!/usr/bin/env python3
"""Device-to-host copy engines and host buffer kinds (an experiment for DESIGN.md §6 "PCIe pass"): 65.5 MB
(one batch of compact codes) copied by hipMemcpyAsync on a stream that has run no kernel (the runtime's SDMA
path) and on a stream whose previous command is a kernel (where the runtime may use a blit kernel), into
torch pinned memory, hipHostMalloc (default / coherent / non-coherent / write-combined), and hipHostRegister'ed
malloc memory; idle device.  One JSON line per case (GB/s, median of 7).

    python benchmarks/sdma_probe.py
"""
import ctypes
import json
import sys
import time

import numpy as np


def main():
    import torch
    dev = torch.device("cuda", 0)
    n = 409600 * 80 * 2
    src = torch.empty(n // 2, dtype=torch.int16, device=dev).random_(-30000, 20000)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    bufs = {"torch_pinned": torch.empty(n // 2, dtype=torch.int16).pin_memory().data_ptr()}
    keep = []
    for name, flags in (("hostmalloc_default", 0x0), ("hostmalloc_coherent", 0x40000000),
                        ("hostmalloc_noncoherent", 0x80000000), ("hostmalloc_writecombined", 0x4)):
        p = ctypes.c_void_p()
        if hip.hipHostMalloc(ctypes.byref(p), n, flags) == 0:
            bufs[name] = p.value
    a = np.empty(n, np.uint8)
    a[:] = 1
    keep.append(a)
    if hip.hipHostRegister(a.ctypes.data, n, 0) == 0:
        bufs["host_register"] = a.ctypes.data
    for after_kernel in (False, True):
        for name, hp in bufs.items():
            for direction in ("d2h", "h2d"):
                rates = []
                for r in range(8):
                    s = torch.cuda.Stream(dev)  # a fresh stream per copy: no earlier command on it
                    with torch.cuda.stream(s):
                        if after_kernel:
                            torch.cuda._sleep(1000)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        if direction == "d2h":
                            rc = hip.hipMemcpyAsync(hp, src.data_ptr(), n, 2, ctypes.c_void_p(s.cuda_stream))
                        else:
                            rc = hip.hipMemcpyAsync(src.data_ptr(), hp, n, 1, ctypes.c_void_p(s.cuda_stream))
                        assert rc == 0
                        e1.record(s)
                    t0 = time.perf_counter()
                    torch.cuda.synchronize(dev)
                    wall = time.perf_counter() - t0
                    if r:
                        rates.append(n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
                rates.sort()
                print(json.dumps(dict(buffer=name, direction=direction, after_kernel=after_kernel,
                                      GBps=round(rates[len(rates) // 2], 1), GBps_min=round(rates[0], 1))), flush=True)


if __name__ == "__main__":
    main()
