"""Executors of a Forest replay (tigerbeetle_amd/forest.py) for tests and the
bench's CPU baseline: the CPU oracle, and a lockstep pair that runs every
batch on the GPU and the oracle and compares them byte for byte.

TEST INFRASTRUCTURE: imports the oracle (the checker), never shipped.
"""
from __future__ import annotations

import time

import numpy as np

from tigerbeetle_amd import trees
from tigerbeetle_amd.tables import TableInfo


class _Result:
    def __init__(self, o):
        self.status = o.status
        self.value_count = o.value_count
        self.data_block_count = o.data_block_count
        self.table_count = len(o.table_infos)
        self.block_count = len(o.blocks)


class OracleManifestStore:
    """Manifest blocks closed by the oracle's restatement of close_block
    (oracle.manifest_blocks) into the executor's host grid."""

    def __init__(self, oracle, grid: dict, cluster: int, block_size: int):
        self.oracle, self.grid, self.cluster, self.bs = oracle, grid, cluster, block_size
        self.checksums: dict = {}
        self.closed: list = []

    def close(self, infos, address, previous_address):
        prev = self.checksums[previous_address] if previous_address else 0
        imgs, sums = self.oracle.manifest_blocks(infos, [address], self.cluster, self.bs, previous_checksum=prev,
                                                 previous_address=previous_address)
        assert len(imgs) == 1
        self.grid[int(address)] = imgs[0]
        self.checksums[int(address)] = sums[0]
        self.closed.append(int(address))

    def read(self, address):
        return self.grid[int(address)]

    def checksum(self, address):
        return self.checksums[int(address)]


class LockstepManifestStore:
    """Every manifest block closed on the GPU grid and by the oracle; reads
    return the GPU's block after comparing it with the oracle's."""

    def __init__(self, gpu_store, ref_store):
        self.gpu, self.ref = gpu_store, ref_store
        self.compared = 0

    def close(self, infos, address, previous_address):
        self.gpu.close(infos, address, previous_address)
        self.ref.close(infos, address, previous_address)

    def checksum(self, address):
        got, want = self.gpu.checksum(address), self.ref.checksum(address)
        assert got == want, f"manifest block {address} checksum"
        return got

    def restore_link(self, address, checksum):
        self.gpu.restore_link(address, checksum)

    def read(self, address):
        got = self.gpu.read(address)
        want = self.ref.read(address)
        assert np.array_equal(got, want), f"manifest block {address}"
        self.compared += 1
        return got

    def check_all(self) -> int:
        """Every block closed so far, GPU grid vs oracle, byte for byte."""
        assert self.gpu.closed == self.ref.closed
        if not self.gpu.closed:
            return 0
        got = self.gpu.grid.get_blocks(self.gpu.closed)
        for a, g in zip(self.gpu.closed, got):
            w = self.ref.grid[a]
            assert np.array_equal(g[:len(w)], w), f"manifest block {a}"
        return len(self.gpu.closed)


class OracleExecutor:
    """The oracle on a host grid (address -> block image), memtables as
    numpy arrays. `busy` accumulates the time spent inside the oracle's sort
    and compaction calls (the CPU baseline's clock)."""

    def __init__(self, oracle, block_size: int = 1 << 20):
        self.oracle, self.bs = oracle, block_size
        self.grid: dict = {}
        self.mutable: dict = {}
        self.immutable: dict = {}
        self.busy = 0.0
        self.input_bytes = 0
        self.last: list = []

    def manifest_store(self, cluster):
        return OracleManifestStore(self.oracle, self.grid, cluster, self.bs)

    def _tree(self, spec):
        return self.oracle.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                                spec.value_count_max, self.bs)

    def put(self, name, values):
        self.mutable.setdefault(name, []).append(np.ascontiguousarray(values))

    def swap(self, names):
        """Every memtable becomes immutable (one run of values); the ones
        named are sorted (TableMemory.sort, table_memory.zig:140-150)."""
        for name in set(self.mutable) | set(self.immutable):
            vals = self.mutable.get(name, [])
            self.mutable[name] = []
            self.immutable[name] = [np.concatenate(vals)] if vals else []
        for name in names:
            spec = trees.BY_NAME[name]
            if not self.immutable[name]:
                continue
            t0 = time.perf_counter()
            self.immutable[name] = [self.oracle.sort_values(self._tree(spec), self.immutable[name][0])]
            self.busy += time.perf_counter() - t0

    def flushed(self, name):
        pass

    def restart(self):
        self.mutable, self.immutable = {}, {}

    def table_segments(self, info: TableInfo, spec) -> list:
        """A table's data blocks' values, found through its index block
        (TableIndex.data_addresses, schema.zig:80-260)."""
        lay = spec.layout(self.bs)
        vcm, dbcm, ks = lay["block_value_count_max"], lay["data_block_count_max"], spec.key_size
        index = self.grid[info.address]
        addr_off = 256 + dbcm * (32 + 2 * ks)
        nblk = -(-info.value_count // vcm)
        segs = []
        for k in range(nblk):
            a = int(index[addr_off + 8 * k:addr_off + 8 * k + 8].view(np.uint64)[0])
            blk = self.grid[a]
            n = int(blk[132:136].view(np.uint32)[0])
            segs.append(blk[256:256 + n * spec.value_size].reshape(n, spec.value_size))
        return segs

    def run_job(self, name, c, cluster):
        spec = c.tree
        if c.table_a is None:
            segs_a = [v for v in self.immutable[name] if len(v)]
        else:
            segs_a = self.table_segments(c.table_a, spec)
        segs_b = [s for t in c.range_b[2] for s in self.table_segments(t, spec)]
        self.input_bytes += sum(s.nbytes for s in segs_a) + sum(s.nbytes for s in segs_b)
        t0 = time.perf_counter()
        o = self.oracle.compact(self._tree(spec), segs_a, segs_b, a_immutable=c.table_a is None,
                                drop_tombstones=c.drop_tombstones, level_b=c.level_b, cluster=cluster,
                                snapshot_min=c.snapshot_min, addresses=c.addresses)
        self.busy += time.perf_counter() - t0
        assert o.status == 0, (name, o.status)
        for a, blk in zip(c.addresses, o.blocks):
            # the on-disk image only (grid.zig:686): a whole replay's blocks stay resident
            size = int(blk[96:100].view(np.uint32)[0])
            self.grid[int(a)] = blk[:size].copy()
        return o

    def submit(self, jobs, cluster):
        return [(c, self.run_job(name, c, cluster)) for name, c in jobs]

    def wait(self, handle, compactions):
        for (c0, o), c in zip(handle, compactions):
            assert c0 is c
            c.result = _Result(o)
            c.outputs = [TableInfo.decode(raw, c.tree.key_size) for raw in o.table_infos]


class LockstepExecutor:
    """Every batch on the GPU grid executor and on the oracle; each job's
    results, TableInfos and output blocks (on-disk images) must be equal."""

    def __init__(self, gpu, oracle_exec: OracleExecutor):
        self.gpu, self.ref = gpu, oracle_exec
        self.jobs_checked = 0
        self.blocks_checked = 0

    def manifest_store(self, cluster):
        self.manifest = LockstepManifestStore(self.gpu.manifest_store(cluster), self.ref.manifest_store(cluster))
        return self.manifest

    def put(self, name, values):
        self.gpu.put(name, values)
        self.ref.put(name, values)

    def swap(self, names):
        self.gpu.swap(names)
        self.ref.swap(names)

    def flushed(self, name):
        self.gpu.flushed(name)

    def checkpoint(self):
        self.gpu.checkpoint()

    def restart(self):
        self.gpu.restart()
        self.ref.restart()

    def submit(self, jobs, cluster):
        return (self.gpu.submit(jobs, cluster), self.ref.submit(jobs, cluster), [name for name, _ in jobs])

    def wait(self, handle, compactions):
        from helpers import disk_image
        h_gpu, h_ref, names = handle
        self.gpu.wait(h_gpu, compactions)
        for (c, o), name in zip(h_ref, names):
            r = c.result
            assert (r.status, r.value_count, r.block_count) == (0, o.value_count, len(o.blocks)), name
            want = [TableInfo.decode(raw, c.tree.key_size) for raw in o.table_infos]
            assert c.outputs == want, name
            got = self.gpu.grid.get_blocks(c.addresses[:r.block_count])
            for g, w in zip(got, o.blocks):
                assert np.array_equal(disk_image(g), disk_image(w)), (name, c.level_b)
            self.jobs_checked += 1
            self.blocks_checked += len(o.blocks)
