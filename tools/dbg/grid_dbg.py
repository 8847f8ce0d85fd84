"""Step-by-step run of the grid test body with progress prints (debug)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
from oracle import oracle
from tigerbeetle_amd import Engine, Grid, Job, Memtable, abi, trees, workloads
import test_gpu_grid as T

def log(*a):
    print(time.strftime("%H:%M:%S"), *a, flush=True)

oracle.build()
eng = Engine(device=0, block_size=1 << 20, profile=True)
log("engine")
rng = np.random.default_rng(1)
grid = Grid(eng, 100)
spec = trees.BY_NAME["transfers.id"]
vals = T.sorted_unique(spec, 50_000, rng)
blocks, ti = T.storage_table(oracle, spec, vals, np.arange(1, 10, dtype=np.uint64))
log("storage table", len(blocks), ti)
grid.put_blocks(np.arange(1, 1 + len(blocks), dtype=np.uint64), np.stack(blocks))
eng.synchronize()
log("put done")
got = grid.get_blocks(np.arange(1, 1 + len(blocks), dtype=np.uint64))
log("get done", all(np.array_equal(g, b[:len(g)]) or np.array_equal(g[:len(b)], b) for g, b in zip(got, blocks)))
mode = sys.argv[1] if len(sys.argv) > 1 else "disk"
if mode == "disk":
    job = Job(spec, [], [], False, False, 2, T.CLUSTER, 48, np.arange(50, 59, dtype=np.uint64), None,
              flags=abi.COMPACTION_GRID, grid=grid, tables_a=[ti.ref()])
else:
    m = Memtable(eng, spec)
    m.put(vals[:1000])
    p, n = m.values()
    job = Job(spec, [(p, n)], [], True, False, 2, T.CLUSTER, 48, np.arange(50, 59, dtype=np.uint64), None,
              flags=abi.COMPACTION_GRID, grid=grid, tables_b=[ti.ref()])
b = eng.submit([job])
log("submitted")
for i in range(200):
    st = b.poll()
    if st != abi.TBC_PENDING:
        break
    time.sleep(0.05)
log("poll", st)
if st != abi.TBC_PENDING:
    r, inf = b.result(0)
    log("result", r.status, r.value_count, r.block_count, b.kernel_times())
    b.release()
log("end")
os._exit(0)
