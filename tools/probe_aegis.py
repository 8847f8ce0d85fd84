"""Probe: AEGIS-128L checksum kernel latency/throughput on N 1-MiB messages."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tigerbeetle_amd import Engine

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
L = 1048320
with Engine(device=0) as e:
    buf = e.alloc(n * (1 << 20))
    rng = np.random.default_rng(1)
    chunk = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    for i in range(n):
        buf.upload(chunk, i * (1 << 20))
    ptrs = [buf.ptr + i * (1 << 20) for i in range(n)]
    for k in [1, 64, n]:
        e.checksum_device(ptrs[:k], [L] * k)
        t0 = time.perf_counter()
        e.checksum_device(ptrs[:k], [L] * k)
        dt = time.perf_counter() - t0
        print(f"messages={k:5d} time={dt*1e3:8.3f} ms  per-update={dt/32767*1e9:7.1f} ns  "
              f"throughput={k*L/dt/1e9:8.2f} GB/s", flush=True)
