"""Host-side anatomy of a bench step (submit call, wait, release) for two arena sizes."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from tigerbeetle_amd import Engine
for arena in (0, 2 << 30):
    eng = Engine(device=0, block_size=1 << 20, profile=True, arena_bytes=arena)
    wl = bench.Workload(eng, 2, list(range(28)), 1 << 20)
    eng.synchronize()
    for _ in range(3):
        wl.step(eng).release()
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        b = eng.submit(wl.jobs)
        t1 = time.perf_counter()
        b.wait()
        t2 = time.perf_counter()
        kt = b.kernel_times()
        b.release()
        t3 = time.perf_counter()
        ts.append((t1 - t0, t2 - t1, t3 - t2, sum(kt.values()) * 1e-6))
    import numpy as np
    m = np.median(np.array(ts), axis=0) * 1e3
    print(" ".join(f"{(a+b+c)*1e3:.2f}" for a, b, c, _ in ts))
    print(f"arena={arena>>20} MiB submit {m[0]:.3f} ms wait {m[1]:.3f} ms release {m[2]:.3f} ms kernels {m[3]:.3f} ms", flush=True)
    eng.close()
