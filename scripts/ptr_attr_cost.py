#!/usr/bin/env python3
"""Cost of hipPointerGetAttributes on this box (the runtime asks it per image
to tell device from host buffers)."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
x = [torch.empty(25 << 20, dtype=torch.uint8, device="cuda") for _ in range(64)]
torch.cuda.synchronize()
attr = ctypes.create_string_buffer(256)
for label, ptrs in (("device", [t.data_ptr() for t in x]),
                    ("host", [ctypes.addressof(ctypes.create_string_buffer(64)) for _ in range(64)])):
    t0 = time.perf_counter()
    n = 0
    for _ in range(50):
        for p in ptrs:
            hip.hipPointerGetAttributes(attr, ctypes.c_void_p(p))
            n += 1
    dt = time.perf_counter() - t0
    print(f"{label}: {dt / n * 1e6:.2f} us per call ({n} calls, ctypes overhead included)")
t0 = time.perf_counter()
for _ in range(3200):
    hip.hipGetLastError()
print(f"ctypes floor (hipGetLastError): {(time.perf_counter() - t0) / 3200 * 1e6:.2f} us")
