"""Benchmark: GPU LSM compaction throughput (BASELINE.json metric).

Default workload (BASELINE.json configs[1]):
transfers id-tree L0->L1 compaction, 28 independent jobs per GPU. Each job
draws 2,358,720 unique uniform-random u128 ids (seed 0x7B0002 + job);
262,080 of them form table A (one level-0 disk table), the rest are sorted
and cut into 8 full level-B tables. IdTreeValue{id, timestamp, padding = 0},
no tombstones, drop_tombstones = false, usage general. 66,044,160 values x
32 B = 2.11 GB of input per GPU, resident in HBM (as 1 MiB grid blocks)
before timing. `--config 3|4|5` run BASELINE configs[2] / [3] / [4]
(tigerbeetle_amd/configs.py); config 3's step includes landing each unsorted
memtable (a D2D copy) and sorting all of them (tbc_sort_values_batch).

A step = one batch of all the GPU's compactions (merge, data blocks with
AEGIS-128L checksums, index blocks, TableInfos) through the C ABI. Multi-GPU:
every rank compacts its own jobs (jobs shard with no data-path collective:
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

from tigerbeetle_amd import Engine, Job, configs  # noqa: E402
from tigerbeetle_amd.shard import plan_shards, reduce_step  # noqa: E402

METRIC = "compacted input MB/s per GPU and per node (1/2/4/8) + % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def blocks_of(table: np.ndarray, vcm: int) -> list:
    return [table[i:i + vcm] for i in range(0, len(table), vcm)]


class Workload:
    """All jobs of one GPU staged in HBM: disk tables as 1 MiB grid blocks,
    memtables as one contiguous array (plus the unsorted copy they are
    re-landed from each step when the config sorts them)."""

    def __init__(self, eng: Engine, config: int, job_ids: list, bs: int):
        self.config = config
        self.bs = bs
        self.jobs, self.bufs, self.specs = [], [], []
        self.sorts, self.landings = [], []
        self.input_values = 0
        self.input_bytes = 0
        self.sort_bytes = 0
        base_addr = 1
        for gid in job_ids:
            js = configs.GENERATORS[config](gid)
            spec = js.tree
            lay = spec.layout(bs)
            vcm = lay["block_value_count_max"]
            reservation = (len(js.b_tables) + 1) * lay["block_count_max"]  # compaction.zig:316-318
            if js.a_immutable:
                abuf = eng.upload(js.a) if len(js.a) else None
                segs_a = [(abuf.ptr, len(js.a))] if abuf else []
                if abuf:
                    self.bufs.append(abuf)
                if js.a_unsorted:
                    pristine = eng.upload(js.a)
                    self.bufs.append(pristine)
                    self.landings.append((abuf.ptr, pristine.ptr, js.a.nbytes))
                    self.sorts.append((spec, abuf.ptr, len(js.a)))
                    self.sort_bytes += 2 * js.a.nbytes
                tables = []
            else:
                tables = [blocks_of(js.a, vcm)]
                segs_a = None
            tables += [blocks_of(t, vcm) for t in js.b_tables]
            nblk = sum(len(t) for t in tables)
            segs = []
            if nblk:
                host = np.zeros((nblk, bs), dtype=np.uint8)
                k = 0
                for t in tables:
                    for v in t:
                        host[k, 256:256 + v.nbytes] = v.reshape(-1)
                        segs.append((k, len(v)))
                        k += 1
                ibuf = eng.upload(host)
                del host
                self.bufs.append(ibuf)
                seg_ptrs = [(ibuf.ptr + i * bs + 256, c) for i, c in segs]
            else:
                seg_ptrs = []
            if segs_a is None:
                na = len(tables[0])
                segs_a, segs_b = seg_ptrs[:na], seg_ptrs[na:]
            else:
                segs_b = seg_ptrs
            out = eng.alloc(reservation * bs)
            addrs = np.arange(base_addr, base_addr + reservation, dtype=np.uint64)
            base_addr += reservation
            self.jobs.append(Job(spec, segs_a, segs_b, js.a_immutable, js.drop_tombstones, js.level_b, 0xA5A5, 48,
                                 addrs, out))
            self.specs.append(js)
            self.bufs.append(out)
            self.input_values += js.input_values
            self.input_bytes += js.input_bytes
            del js

    def step(self, eng: Engine):
        """One step: land + sort the bar's memtables (config 3), then the
        compaction batch; returns the completed batch."""
        for dst, src, n in self.landings:
            eng.copy_device_async(dst, src, n)
        if self.sorts:
            eng.sort_values_batch(self.sorts)
        b = eng.submit(self.jobs)
        b.wait()
        return b


def cpu_baseline(config: int, njobs: int, budget_s: float = 12.0, bs: int = 1 << 20) -> dict:
    """The oracle (single-threaded C restatement, AES-NI AEGIS) on a bounded
    sample of the same workload: whole jobs (memtable sort included for
    config 3) until the time budget is used."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle
    oracle.build()
    total_bytes, total_t, jobs = 0, 0.0, 0
    while total_t < budget_s and jobs < njobs:
        js = configs.GENERATORS[config](jobs)
        spec = js.tree
        t = oracle.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                        spec.value_count_max, bs)
        vcm = t.block_value_count_max
        segs_b = [blk for tb in js.b_tables for blk in blocks_of(tb, vcm)]
        reservation = (len(js.b_tables) + 1) * (t.data_block_count_max + 1)
        t0 = time.perf_counter()
        a = oracle.sort_values(t, js.a) if js.a_unsorted else js.a
        segs_a = ([a] if len(a) else []) if js.a_immutable else blocks_of(a, vcm)
        r = oracle.compact(t, segs_a, segs_b, a_immutable=js.a_immutable, drop_tombstones=js.drop_tombstones,
                           level_b=js.level_b, cluster=0xA5A5, snapshot_min=48,
                           addresses=np.arange(1, 1 + reservation, dtype=np.uint64))
        total_t += time.perf_counter() - t0
        assert r.status == 0
        total_bytes += js.input_bytes
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
            "sample": f"{jobs} of {njobs} jobs ({total_bytes/1e6:.0f} MB of input) of config {config} through "
                      f"oracle/tbc_oracle.c (single thread, AES-NI={bool(olib().tbo_has_aesni())}) on {cpu}"}


# bench kernel label -> rocprofv3 kernel symbol (tools/traffic.py short names)
KERNEL_SYMBOL = {"merge_partition": "k_partition_all", "merge": "k_merge_tile", "data_blocks": "k_data_blocks",
                 "assemble": "k_assemble",
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(configs.GENERATORS))
    ap.add_argument("--jobs", type=int, default=None, help="jobs per GPU (default: the config's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    njobs = args.jobs or configs.DEFAULT_JOBS[args.config]

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for a 1-GPU box (the driver's N>1 runs use neither):
    # every rank on device 0, timing reduction over gloo.
    if os.environ.get("TBC_BENCH_SAME_DEVICE"):
        local = 0
    backend = os.environ.get("TBC_BENCH_BACKEND", "nccl")  # nccl = RCCL over xGMI
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group(backend)
        dist = td

    bs = 1 << 20
    eng = Engine(device=local, block_size=bs, profile=True, arena_bytes=2 << 30)
    # Weak scaling: njobs jobs per GPU; the global job set is sharded by
    # input bytes (LPT, shard.py), no data-path collective.
    plan = plan_shards([configs.job_bytes(args.config, j) for j in range(njobs * world)], world)
    wl = Workload(eng, args.config, plan[rank], bs)
    eng.synchronize()

    for _ in range(args.warmup):
        wl.step(eng).release()

    def barrier():
        eng.synchronize()
        if dist:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    import gc
    gc.collect()
    gc.disable()  # no collector pause inside the timed region
    t0 = time.perf_counter()
    ktimes: dict = {}
    marks = []
    for _ in range(args.steps):
        b = wl.step(eng)
        marks.append(time.perf_counter())
        for k, v in b.kernel_times().items():
            ktimes[k] = ktimes.get(k, 0.0) + v
        b.release()
    barrier()
    gc.enable()
    if os.environ.get("TBC_BENCH_TRACE"):
        print("step ms:", " ".join(f"{(b - a) * 1e3:.2f}" for a, b in zip([t0] + marks, marks)), file=sys.stderr)
    dt = time.perf_counter() - t0
    # Check the last step's results: every job OK, and output shape for the bytes.
    b = wl.step(eng)
    out_values = data_blocks = tables = index_bytes = 0
    for i, js in enumerate(wl.specs):
        r, _ = b.result(i)
        assert r.status == 0, (i, r.status)
        out_values += r.value_count * js.tree.value_size
        data_blocks += r.data_block_count
        tables += r.table_count
        index_bytes += r.table_count * js.tree.layout(bs)["index_size"]
        if args.config == 2 and not os.environ.get("TBC_LIB"):  # ablation builds (timing only) skip this
            assert r.value_count == 9 * configs.TABLE_T and r.table_count == 9, (r.value_count, r.table_count)
    b.release()

    total_bytes, t_max = reduce_step(dist, wl.input_bytes, dt,
                                     device=f"cuda:{local}" if dist and backend == "nccl" else None)
    step_s = t_max / args.steps
    value = total_bytes / step_s / 1e6

    # Per-kernel device times (hipEvents on the engine's stream), per step.
    per_step = {k: v / args.steps for k, v in ktimes.items()}
    dominant = max(per_step, key=per_step.get)
    R = wl.input_bytes
    W_data = out_values + data_blocks * 256  # out_values is in bytes here
    W_index = index_bytes
    alg_bytes = {
        "merge_partition": len(wl.jobs) * 2400 * 2 * 21 * 32,
        "merge": R,  # read every input value once (keys decide; 2 mask bits per position written)
        "data_blocks": out_values + W_data,  # read every survivor once, write the blocks
        "assemble": 2 * out_values,  # two-pass regime: gather survivors into the bodies
        "index_blocks": W_index + data_blocks * 64,
    }
    if "assemble" in per_step:  # two-pass regime: the chains read the assembled bodies and write headers
        alg_bytes["data_blocks"] = out_values + data_blocks * 256
    kt_us = per_step[dominant]
    achieved = alg_bytes.get(dominant, R) / (kt_us * 1e-6) / 1e9
    job_bytes = R + W_data + W_index + wl.sort_bytes  # R + W (+ S)
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
        "data": f"synthetic (seeded tables, BASELINE config {args.config}: tigerbeetle_amd/configs.py)",
        "config": {"workload": configs.DESCRIPTION[args.config], "baseline_config": args.config,
                   "jobs_per_gpu": njobs, "input_bytes_per_gpu": wl.input_bytes, "block_size": bs,
                   "parallelism": f"shard-by-job x{world}"},
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": alg_bytes.get(dominant, R)},
        "job_roofline": {"bytes": job_bytes, "achieved": round(job_bytes / step_s / 1e9, 1), "unit": "GB/s",
                         "frac": round(job_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4)},
        "kernels_us_per_step": {k: round(v, 1) for k, v in per_step.items()},
    }
    if "assemble" not in per_step and "data_blocks" in per_step:
        # Latency regime: every data block's AEGIS-128L chain is in flight at
        # once, so the data-block kernel is bound by the chain of the longest
        # block (32,767 sequential updates for a full 1 MiB body), not by HBM.
        # Floor: 58.3 ns per update for one chain alone on an idle MI355X
        # (tools/chain_probe.py).
        updates = (bs - 256 + 31) // 32 + 7
        floor_us = updates * 58.3e-3
        line["latency_roofline"] = {"bound": "aegis_chain", "kernel": "data_blocks",
                                    "updates_per_block": updates, "floor_us": round(floor_us, 1),
                                    "achieved_us": round(per_step["data_blocks"], 1),
                                    "frac": round(floor_us / per_step["data_blocks"], 4)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.config, njobs)
    if rank == 0:
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
