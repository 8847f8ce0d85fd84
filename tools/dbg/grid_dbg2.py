"""Replay of test_two_half_bars_chained_through_the_grid with stage syncs (debug)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
from oracle import oracle
from tigerbeetle_amd import Engine, Grid, Job, Memtable, abi, trees, workloads
from tigerbeetle_amd.tables import TableInfo
import test_gpu_grid as T

def log(*a):
    print(time.strftime("%H:%M:%S"), *a, flush=True)

oracle.build()
engine = Engine(device=0, block_size=1 << 20, profile=True)
oracle_lib = oracle
rng = np.random.default_rng(0x6A1D)
grid = Grid(engine, 600)
spec_id = trees.BY_NAME["transfers.id"]
universe = T.sorted_unique(spec_id, 160_000, rng)
pick = np.zeros(len(universe), bool)
pick[rng.choice(len(universe), 90_000, replace=False)] = True
b_all = universe[~pick]
b1, b2 = b_all[: len(b_all) // 2], b_all[len(b_all) // 2:]
blk1, ti1 = T.storage_table(oracle_lib, spec_id, b1, np.arange(1, 20, dtype=np.uint64), level=0)
blk2, ti2 = T.storage_table(oracle_lib, spec_id, b2, np.arange(20, 40, dtype=np.uint64), level=0)
for blocks, ti, base in ((blk1, ti1, 1), (blk2, ti2, 20)):
    grid.put_blocks(np.arange(base, base + len(blocks), dtype=np.uint64), np.stack(blocks))
mem_vals = universe[pick]
shuffled = workloads.shuffle_for_memtable(mem_vals, rng, spec_id)
mem = Memtable(engine, spec_id)
for lo in range(0, len(shuffled), 8190):
    mem.put(shuffled[lo:lo + 8190])
mptr, mcount = mem.values()
engine.sort_values_batch([(spec_id, mptr, mcount)])
a1 = np.arange(100, 100 + 3 * 9, dtype=np.uint64)
b = engine.submit([Job(spec_id, [(mptr, mcount)], [], True, False, 0, T.CLUSTER, 48, a1, None,
                       flags=abi.COMPACTION_GRID, grid=grid, tables_b=[ti1.ref(), ti2.ref()])])
b.wait()
r1, inf1 = b.result(0)
b.release()
log("batch1", r1.status, r1.value_count, r1.block_count)
out_t0 = TableInfo.decode(inf1[0], spec_id.key_size)
log("out_t0", out_t0)
more = T.sorted_unique(spec_id, 40_000, rng)
blk5, ti5 = T.storage_table(oracle_lib, spec_id, more, np.arange(300, 320, dtype=np.uint64), level=1)
log("ti5", ti5, len(blk5))
grid.put_blocks(np.arange(300, 300 + len(blk5), dtype=np.uint64), np.stack(blk5))
engine.synchronize()
mode = sys.argv[1] if len(sys.argv) > 1 else "both"
ta = [out_t0.ref()] if mode in ("both", "a") else []
tb = [ti5.ref()] if mode in ("both", "b") else []
a3 = np.arange(400, 400 + 2 * 9, dtype=np.uint64)
b = engine.submit([Job(spec_id, [], [], False, False, 1, T.CLUSTER, 64, a3, None, flags=abi.COMPACTION_GRID,
                       grid=grid, tables_a=ta, tables_b=tb)])
log("submitted 2")
st = None
for i in range(100):
    st = b.poll()
    if st != abi.TBC_PENDING:
        break
    time.sleep(0.05)
log("poll", st)
if st not in (abi.TBC_PENDING, abi.TBC_ERR_DEVICE):
    r, inf = b.result(0)
    log("result", r.status, r.value_count, r.block_count)
os._exit(0)
