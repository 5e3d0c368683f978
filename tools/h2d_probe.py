"""H2D bandwidth from pinned (hipHostMalloc) and registered (hipHostRegister) host memory,
one stream vs several concurrent streams (64 MiB pieces)."""
import ctypes, os, sys, time
import numpy as np
import torch
sys.path.insert(0, '.')
n = 800 << 20
piece = 64 << 20
d = torch.empty(n, dtype=torch.uint8, device="cuda")


def run(h, label):
    for ns in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        for rep in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i, off in enumerate(range(0, n, piece)):
                with torch.cuda.stream(streams[i % ns]):
                    d[off:off + piece].copy_(h[off:off + piece], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        print(f"{label} streams={ns}: {n / dt / 1e9:.1f} GB/s", flush=True)


run(torch.empty(n, dtype=torch.uint8).pin_memory(), "hipHostMalloc")
import pktvisor_amd as pa
lib = pa.load_library()
a = np.ones(n, dtype=np.uint8)
assert lib.pv_host_register(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(n)) == 0
run(torch.from_numpy(a), "hipHostRegister")
