"""AEGIS chain throughput vs in-flight messages: tbc_checksum_batch over n x 1 MiB bodies."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tigerbeetle_amd import Engine
eng = Engine(device=0, block_size=1 << 20)
L = (1 << 20) - 256
n_max = 13824
buf = eng.alloc(n_max * (1 << 20))
buf.zero()
for n in (1, 2016, 4096, 8192, 13824):
    ptrs = [buf.ptr + i * (1 << 20) for i in range(n)]
    lens = [L] * n
    eng.checksum_device(ptrs, lens)
    t = time.perf_counter()
    eng.checksum_device(ptrs, lens)
    dt = time.perf_counter() - t
    print(f"{n:6d} messages: {dt*1e3:8.2f} ms  {n*L/dt/1e9:8.1f} GB/s  {dt/32767*1e9:6.1f} ns/update", flush=True)
