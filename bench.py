"""Benchmark: GPU LSM compaction throughput (BASELINE.json metric).

Workload (BASELINE.json configs[1]): transfers id-tree
L0->L1 compaction, 28 independent jobs per GPU. Each job draws 2,358,720
unique uniform-random u128 ids (seed 0x7B0002 + job); 262,080 of them form
table A (one level-0 disk table), the rest are sorted and cut into 8 full
level-B tables. IdTreeValue{id, timestamp, padding = 0}, no tombstones,
drop_tombstones = false, usage general. 66,044,160 values x 32 B = 2.11 GB of
input per GPU, resident in HBM (as 1 MiB grid blocks) before timing.

A step = one batch of all 28 compactions (merge, data blocks with AEGIS-128L
checksums, index blocks, TableInfos) through the C ABI. Multi-GPU: every
rank compacts its own 28 jobs (jobs shard with no data-path collective:
weak scaling); value = total input bytes of all ranks / max-over-ranks time.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tigerbeetle_amd import Engine, Job, trees  # noqa: E402
from tigerbeetle_amd.shard import plan_shards, reduce_step  # noqa: E402

METRIC = "compacted input MB/s per GPU and per node (1/2/4/8) + % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
TABLE = 262_080
JOBS = 28
SEED = 0x7B0002


def gen_job(job: int, n_b_tables: int = 8):
    """Values of one L0->L1 id-tree compaction: A (1 table) and B (8 tables)."""
    rng = np.random.default_rng(SEED + job)
    n = TABLE * (n_b_tables + 1)
    hi = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n, dtype=np.uint64)
    lo = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n, dtype=np.uint64)
    order = np.lexsort((lo, hi))
    hi, lo = hi[order], lo[order]
    dup = (hi[1:] == hi[:-1]) & (lo[1:] == lo[:-1])
    assert not dup.any(), "duplicate u128 id drawn"
    vals = np.zeros((n, 32), dtype=np.uint8)
    w = vals.view(np.uint64)
    w[:, 0] = lo
    w[:, 1] = hi
    w[:, 2] = rng.permutation(n).astype(np.uint64) + np.uint64(1)  # timestamps, insertion order
    a_idx = np.sort(rng.choice(n, size=TABLE, replace=False))
    mask = np.zeros(n, dtype=bool)
    mask[a_idx] = True
    a = vals[mask]
    b = vals[~mask]
    return a, [b[i * TABLE:(i + 1) * TABLE] for i in range(n_b_tables)]


def blocks_of(table: np.ndarray, vcm: int) -> list:
    return [table[i:i + vcm] for i in range(0, len(table), vcm)]


class Workload:
    """All jobs of one GPU staged in HBM as 1 MiB grid blocks."""

    def __init__(self, eng: Engine, job_ids: list, bs: int):
        self.spec = trees.BY_NAME["transfers.id"]
        self.bs = bs
        lay = self.spec.layout(bs)
        self.vcm = lay["block_value_count_max"]
        self.block_count_max = lay["block_count_max"]
        self.jobs, self.bufs = [], []
        self.input_values = 0
        for j, gid in enumerate(job_ids):
            a, b_tables = gen_job(gid)
            tables = [blocks_of(a, self.vcm)] + [blocks_of(t, self.vcm) for t in b_tables]
            nblk = sum(len(t) for t in tables)
            host = np.zeros((nblk, bs), dtype=np.uint8)
            segs, k = [], 0
            for t in tables:
                for v in t:
                    host[k, 256:256 + v.nbytes] = v.reshape(-1)
                    segs.append((k, len(v)))
                    k += 1
            ibuf = eng.upload(host)
            del host
            seg_ptrs = [(ibuf.ptr + i * bs + 256, c) for i, c in segs]
            na = len(blocks_of(a, self.vcm))
            reservation = (len(b_tables) + 1) * self.block_count_max  # compaction.zig:316-318
            out = eng.alloc(reservation * bs)
            addrs = np.arange(1 + j * reservation, 1 + (j + 1) * reservation, dtype=np.uint64)
            self.jobs.append(Job(self.spec, seg_ptrs[:na], seg_ptrs[na:], False, False, 1, 0xA5A5, 48,
                                 addrs, out))
            self.bufs += [ibuf, out]
            self.input_values += len(a) + sum(len(t) for t in b_tables)

    @property
    def input_bytes(self) -> int:
        return self.input_values * self.spec.value_size


def cpu_baseline(budget_s: float = 12.0, bs: int = 1 << 20) -> dict:
    """The oracle (single-threaded C restatement, AES-NI AEGIS) on a bounded
    sample of the same workload: whole jobs until the time budget is used."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle
    oracle.build()
    spec = trees.BY_NAME["transfers.id"]
    t = oracle.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                    spec.value_count_max, bs)
    vcm = t.block_value_count_max
    total_bytes, total_t, jobs = 0, 0.0, 0
    while total_t < budget_s and jobs < JOBS:
        a, b_tables = gen_job(jobs)
        segs_a = blocks_of(a, vcm)
        segs_b = [blk for tb in b_tables for blk in blocks_of(tb, vcm)]
        reservation = (len(b_tables) + 1) * (t.data_block_count_max + 1)
        t0 = time.perf_counter()
        r = oracle.compact(t, segs_a, segs_b, a_immutable=False, drop_tombstones=False, level_b=1, cluster=0xA5A5,
                           snapshot_min=48, addresses=np.arange(1, 1 + reservation, dtype=np.uint64))
        total_t += time.perf_counter() - t0
        assert r.status == 0
        total_bytes += (len(a) + sum(len(x) for x in b_tables)) * spec.value_size
        jobs += 1
    import platform
    cpu = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    from oracle.oracle import lib as olib
    return {"value": round(total_bytes / total_t / 1e6, 1), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": f"{jobs} of {JOBS} jobs ({total_bytes/1e6:.0f} MB of input) through oracle/tbc_oracle.c "
                      f"(single thread, AES-NI={bool(olib().tbo_has_aesni())}) on {cpu}"}


# bench kernel label -> rocprofv3 kernel symbol (tools/traffic.py short names)
KERNEL_SYMBOL = {"merge_partition": "k_partition", "merge": "k_merge_tile", "data_blocks": "k_data_blocks",
                 "index_blocks": "k_index_blocks"}


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the PMC passes committed under
    profiles/*/traffic.json (tools/profile.sh + tools/traffic.py), used only
    when that profile was taken with this very libtbc.so (md5 match)."""
    import glob
    import hashlib
    from tigerbeetle_amd import abi
    try:
        md5 = hashlib.md5(open(abi.LIB_PATH, "rb").read()).hexdigest()
    except OSError:
        return None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json"))):
        d = json.load(open(f))
        k = d.get("kernels", {}).get(KERNEL_SYMBOL.get(kernel, kernel))
        if d.get("lib_md5") == md5 and k:
            return k["traffic_bytes"], os.path.relpath(f, ROOT)
    return None, None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--jobs", type=int, default=JOBS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group("nccl")
        dist = td

    bs = 1 << 20
    eng = Engine(device=local, block_size=bs, profile=True)
    # Weak scaling: args.jobs jobs per GPU; the global job set is sharded by
    # bytes (all jobs are the same size here), no data-path collective.
    plan = plan_shards([1] * (args.jobs * world), world)
    wl = Workload(eng, plan[rank], bs)
    eng.synchronize()

    def step():
        b = eng.submit(wl.jobs)
        b.wait()
        return b

    for _ in range(args.warmup):
        step().release()

    def barrier():
        eng.synchronize()
        if dist:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    ktimes: dict = {}
    for _ in range(args.steps):
        b = step()
        for k, v in b.kernel_times().items():
            ktimes[k] = ktimes.get(k, 0.0) + v
        b.release()
    barrier()
    dt = time.perf_counter() - t0
    # Verify the last step's shape (every job: all values out, 72 data blocks, 9 tables).
    b = step()
    res0, _ = b.result(0)
    b.release()
    if not os.environ.get("TBC_LIB"):  # ablation builds (timing only) skip the shape check
        assert res0.value_count == 9 * TABLE and res0.table_count == 9, (res0.value_count, res0.table_count)

    total_bytes, t_max = reduce_step(dist, wl.input_bytes, dt, device=f"cuda:{local}" if dist else None)
    step_s = t_max / args.steps
    value = total_bytes / step_s / 1e6

    # Per-kernel device times (hipEvents on the engine's stream), per step.
    per_step = {k: v / args.steps for k, v in ktimes.items()}
    dominant = max(per_step, key=per_step.get)
    spec = wl.spec
    n_in = wl.input_values
    out_values = n_in  # no dedup / tombstones in this workload
    data_blocks = args.jobs * 72
    tables = args.jobs * 9
    index_size = spec.layout(bs)["index_size"]
    R = n_in * spec.value_size
    W_data = out_values * spec.value_size + data_blocks * 256
    W_index = tables * index_size
    alg_bytes = {
        "merge_partition": (args.jobs * 2400) * 2 * 21 * 32,
        "merge": R,  # read every input value once (keys decide; 2 mask bits per position written)
        "data_blocks": out_values * spec.value_size + W_data,  # read every survivor once, write the blocks
        "index_blocks": W_index + data_blocks * 64,
    }
    kt_us = per_step[dominant]
    achieved = alg_bytes.get(dominant, R) / (kt_us * 1e-6) / 1e9
    job_bytes = R + W_data + W_index
    traffic, traffic_src = pmc_traffic(dominant)
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "MB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded IdTreeValue tables, config 2)",
        "config": {"workload": "transfers.id L0->L1 compaction, 28 jobs x (1 A + 8 B tables) per GPU, "
                               "64M u128 keys, 1 MiB blocks", "jobs_per_gpu": args.jobs,
                   "input_bytes_per_gpu": wl.input_bytes, "block_size": bs, "parallelism": f"shard-by-job x{world}"},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": alg_bytes.get(dominant, R)},
        "job_roofline": {"bytes": job_bytes, "achieved": round(job_bytes / step_s / 1e9, 1), "unit": "GB/s",
                         "frac": round(job_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4)},
        "kernels_us_per_step": {k: round(v, 1) for k, v in per_step.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
