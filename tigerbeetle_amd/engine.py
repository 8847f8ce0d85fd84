"""Host-side driver of the GPU compaction engine over the C ABI.

`Engine` owns one libtbc engine (a HIP stream plus static device/pinned
arenas) on one GPU. It is the plumbing used by tests and the benchmark; the
production host adapter is the Zig `@cImport` of include/tbc.h (see
INTEGRATION.md) or the C++ mirror in tigerbeetle_amd/host/.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .abi import check, lib
from .trees import BLOCK_SIZE, HEADER_SIZE, TreeSpec


class DeviceBuffer:
    """A device allocation (hipMalloc via tbc_device_alloc)."""

    def __init__(self, engine: "Engine", nbytes: int):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().tbc_device_alloc(engine.handle, max(1, self.nbytes), ctypes.byref(p)), "tbc_device_alloc")
        self.ptr = p.value

    def upload(self, array: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(array)
        assert offset + a.nbytes <= self.nbytes
        check(lib().tbc_copy_to_device(self.engine.handle, self.ptr + offset, a.ctypes.data, a.nbytes),
              "tbc_copy_to_device")

    def download(self, nbytes: int | None = None, offset: int = 0) -> np.ndarray:
        n = self.nbytes - offset if nbytes is None else nbytes
        out = np.empty(n, dtype=np.uint8)
        check(lib().tbc_copy_to_host(self.engine.handle, out.ctypes.data, self.ptr + offset, n),
              "tbc_copy_to_host")
        return out

    def zero(self) -> None:
        check(lib().tbc_memset_device(self.engine.handle, self.ptr, 0, self.nbytes), "tbc_memset_device")

    def free(self) -> None:
        if self.ptr:
            lib().tbc_device_free(self.engine.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr and self.engine.handle:
                self.free()
        except Exception:
            pass


@dataclass
class Job:
    """One Compaction.start(Context) (src/lsm/compaction.zig:84-99)."""
    tree: TreeSpec
    segments_a: list  # [(device_ptr, count)]
    segments_b: list
    a_immutable: bool
    drop_tombstones: bool
    level_b: int
    cluster: int
    snapshot_min: int
    addresses: np.ndarray  # uint64, acquire order
    output: DeviceBuffer
    flags: int = 0  # TBC_COMPACTION_* (abi.COMPACTION_VALUES_ONLY, abi.COMPACTION_GRID, abi.COMPACTION_UNIQUE_KEYS)
    grid: "Grid | None" = None   # COMPACTION_GRID: disk tables by reference, outputs into the grid
    tables_a: list = field(default_factory=list)  # [(index address, index checksum u128, value_count)]
    tables_b: list = field(default_factory=list)
    output_offset: int = 0  # VALUES_ONLY: survivors land at the job's output positions output_offset + i (split.py)
    _keep: list = field(default_factory=list)
    _ctype: object = field(default=None, repr=False)

    def ctype(self) -> abi.Compaction:
        """The tbc_compaction descriptor, built once per Job (segment tables
        filled with numpy, not per-element ctypes stores) and reused by every
        submit: the descriptor is host plumbing, not part of the device step."""
        if self._ctype is not None:
            return self._ctype
        c = abi.Compaction()
        c.tree = self.tree.ctype()
        c.a_immutable = int(self.a_immutable)
        c.drop_tombstones = int(self.drop_tombstones)
        c.level_b = self.level_b
        c.flags = self.flags
        sa, sb = _segment_table(self.segments_a), _segment_table(self.segments_b)
        addrs = np.ascontiguousarray(self.addresses, dtype=np.uint64)
        ra, rb = _table_ref_table(self.tables_a), _table_ref_table(self.tables_b)
        self._keep = [sa, sb, addrs, ra, rb]
        c.segments_a = ctypes.cast(sa.ctypes.data, ctypes.POINTER(abi.Segment))
        c.segment_count_a = len(self.segments_a)
        c.segments_b = ctypes.cast(sb.ctypes.data, ctypes.POINTER(abi.Segment))
        c.segment_count_b = len(self.segments_b)
        if self.flags & abi.COMPACTION_GRID:
            c.grid = self.grid.handle
            c.tables_a = ctypes.cast(ra.ctypes.data, ctypes.POINTER(abi.TableRef))
            c.tables_b = ctypes.cast(rb.ctypes.data, ctypes.POINTER(abi.TableRef))
            c.table_count_a = len(self.tables_a)
            c.table_count_b = len(self.tables_b)
        c.cluster[0] = self.cluster & ((1 << 64) - 1)
        c.cluster[1] = self.cluster >> 64
        c.snapshot_min = self.snapshot_min
        c.addresses = addrs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        c.address_count = len(addrs)
        c.output_blocks = self.output.ptr if self.output is not None else None
        c.output_offset = self.output_offset
        self._ctype = c
        return c


def _segment_table(segments: list) -> np.ndarray:
    """tbc_segment[] as a (n, 2) uint64 array: {values, count | reserved << 32}."""
    t = np.zeros((max(1, len(segments)), 2), dtype=np.uint64)
    if segments:
        t[: len(segments)] = np.asarray(segments, dtype=np.uint64).reshape(-1, 2)
    return t


def _table_ref_table(refs: list) -> np.ndarray:
    """tbc_table_ref[] as a (n, 4) uint64 array: {address, checksum lo, hi, value_count}."""
    t = np.zeros((max(1, len(refs)), 4), dtype=np.uint64)
    for i, (address, checksum, count) in enumerate(refs):
        t[i] = (address, checksum & ((1 << 64) - 1), checksum >> 64, count)
    return t


class Grid:
    """The GPU-resident grid (tbc_grid): blocks of addresses [1, block_count] in HBM."""

    def __init__(self, engine: "Engine", block_count: int):
        self.engine = engine
        self.block_count = int(block_count)
        h = ctypes.c_void_p()
        check(lib().tbc_grid_init(engine.handle, self.block_count, ctypes.byref(h)), "tbc_grid_init")
        self.handle = h.value

    def pointer(self, address: int) -> int:
        p = ctypes.c_void_p()
        check(lib().tbc_grid_block_pointer(self.handle, int(address), ctypes.byref(p)), "tbc_grid_block_pointer")
        return p.value

    def put_blocks(self, addresses, images: np.ndarray) -> None:
        """Stage host block images (n, block_size) uint8 as blocks read from storage."""
        images = np.ascontiguousarray(images, dtype=np.uint8)
        n = len(addresses)
        A = np.ascontiguousarray(addresses, dtype=np.uint64)
        P = (ctypes.c_void_p * max(1, n))(*[images.ctypes.data + i * images.shape[1] for i in range(n)])
        check(lib().tbc_grid_put_blocks(self.handle, A.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), P, n),
              "tbc_grid_put_blocks")

    def get_blocks(self, addresses, out: np.ndarray | None = None) -> np.ndarray:
        """Copy blocks to host images (n, block_size); `out` may be a
        preallocated (e.g. host-registered) array of at least n rows."""
        n = len(addresses)
        if out is None:
            out = np.zeros((max(1, n), self.engine.block_size), dtype=np.uint8)
        assert out.dtype == np.uint8 and out.flags.c_contiguous and out.shape[0] >= n
        assert out.shape[1] == self.engine.block_size
        A = np.ascontiguousarray(addresses, dtype=np.uint64)
        P = (ctypes.c_void_p * max(1, n))(*[out.ctypes.data + i * self.engine.block_size for i in range(n)])
        check(lib().tbc_grid_get_blocks(self.handle, A.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), P, n),
              "tbc_grid_get_blocks")
        return out[:n]

    def manifest_close_status(self) -> None:
        """tbc_manifest_close_status: wait for the manifest closes enqueued on
        this grid; raise TbcError(TBC_ERR_BLOCK_INVALID) once if one refused
        to link onto an untrusted previous block."""
        check(lib().tbc_manifest_close_status(self.handle), "tbc_manifest_close_status")

    def invalidate(self) -> None:
        """tbc_grid_invalidate: a restart's cold cache (every block validated before use)."""
        check(lib().tbc_grid_invalidate(self.handle), "tbc_grid_invalidate")

    def close(self) -> None:
        if self.handle:
            lib().tbc_grid_deinit(self.handle)
            self.handle = None


class Memtable:
    """A TableMemory on the device (tbc_memtable): puts stream in through pinned staging."""

    def __init__(self, engine: "Engine", tree: TreeSpec, capacity: int | None = None):
        self.engine, self.tree = engine, tree
        t = tree.ctype()
        h = ctypes.c_void_p()
        check(lib().tbc_memtable_init(engine.handle, ctypes.byref(t), int(capacity or tree.value_count_max),
                                      ctypes.byref(h)), "tbc_memtable_init")
        self.handle = h.value

    def put(self, values: np.ndarray) -> None:
        v = np.ascontiguousarray(values, dtype=np.uint8)
        assert v.ndim == 2 and v.shape[1] == self.tree.value_size
        check(lib().tbc_memtable_put(self.handle, v.ctypes.data, len(v)), "tbc_memtable_put")

    def values(self):
        p, n = ctypes.c_void_p(), ctypes.c_uint32()
        check(lib().tbc_memtable_values(self.handle, ctypes.byref(p), ctypes.byref(n)), "tbc_memtable_values")
        return p.value, n.value

    def reset(self) -> None:
        check(lib().tbc_memtable_reset(self.handle), "tbc_memtable_reset")

    @staticmethod
    def make_immutable(engine: "Engine", pairs: list) -> None:
        """tbc_memtable_make_immutable: [(mutable, immutable, in_order)] — each
        mutable table's values become its (empty) immutable table's, in key
        order (one out-of-place sort of every table not in order), and the
        mutable tables are emptied."""
        n = len(pairs)
        if not n:
            return
        muts = (ctypes.c_void_p * n)(*[m.handle for m, _, _ in pairs])
        imms = (ctypes.c_void_p * n)(*[im.handle for _, im, _ in pairs])
        order = (ctypes.c_uint8 * n)(*[1 if o else 0 for _, _, o in pairs])
        check(lib().tbc_memtable_make_immutable(engine.handle, muts, imms, ctypes.cast(order, ctypes.c_void_p), n),
              "tbc_memtable_make_immutable")

    def close(self) -> None:
        if self.handle:
            lib().tbc_memtable_deinit(self.handle)
            self.handle = None


class Batch:
    def __init__(self, engine: "Engine", handle: int, jobs: list):
        self.engine, self.handle, self.jobs = engine, handle, jobs

    def poll(self) -> int:
        return lib().tbc_batch_poll(self.handle)

    def wait(self) -> None:
        check(lib().tbc_batch_wait(self.handle), "tbc_batch_wait")

    def result(self, index: int):
        r = abi.CompactionResult()
        check(lib().tbc_batch_result(self.handle, index, ctypes.byref(r), None, 0), "tbc_batch_result")
        infos = np.zeros((max(1, r.table_count), 128), dtype=np.uint8)
        check(lib().tbc_batch_result(self.handle, index, ctypes.byref(r), infos.ctypes.data, r.table_count),
              "tbc_batch_result")
        return r, infos[: r.table_count]

    def check_results(self) -> None:
        """Raise if any compaction of the (complete) batch did not end TBC_OK."""
        for i in range(len(self.jobs)):
            r = abi.CompactionResult()
            check(lib().tbc_batch_result(self.handle, i, ctypes.byref(r), None, 0), "tbc_batch_result")
            check(r.status, f"compaction {i} of the batch")

    def speculation(self, index: int) -> int:
        """abi.SPECULATION_NONE / _HELD / _BROKEN of compaction `index` (tbc_batch_speculation)."""
        out = ctypes.c_uint32()
        check(lib().tbc_batch_speculation(self.handle, index, ctypes.byref(out)), "tbc_batch_speculation")
        return out.value

    def kernel_times(self) -> dict:
        cap = 32
        names = (ctypes.c_char_p * cap)()
        us = (ctypes.c_double * cap)()
        n = ctypes.c_uint32()
        check(lib().tbc_batch_kernel_times(self.handle, names, us, cap, ctypes.byref(n)), "kernel_times")
        out: dict = {}
        for i in range(n.value):
            k = names[i].decode()
            out[k] = out.get(k, 0.0) + us[i]
        return out

    def release(self) -> None:
        if self.handle:
            lib().tbc_batch_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            if self.handle and self.engine.handle:  # a closed engine took its batches' memory with it
                self.release()
        except Exception:
            pass


class KwayMerge:
    """A submitted k-way merge (tbc_kway_*)."""

    def __init__(self, handle):
        self.handle = handle

    def poll(self) -> bool:
        st = lib().tbc_kway_poll(self.handle)
        if st == abi.TBC_PENDING:
            return False
        check(st, "tbc_kway_poll")
        return True

    def wait(self) -> None:
        check(lib().tbc_kway_wait(self.handle), "tbc_kway_wait")

    def count(self) -> int:
        n = ctypes.c_uint64()
        check(lib().tbc_kway_count(self.handle, ctypes.byref(n)), "tbc_kway_count")
        return n.value

    def release(self) -> None:
        if self.handle:
            lib().tbc_kway_release(self.handle)
            self.handle = None


class Engine:
    def __init__(self, device: int = 0, block_size: int = BLOCK_SIZE, arena_bytes: int = 0,
                 profile: bool = False, pipeline: bool | None = None):
        """pipeline: None = the engine decides per UNIQUE_KEYS batch (pipelined
        when an earlier batch is still running), True / False = always / never
        (TBC_CONFIG_PIPELINE / TBC_CONFIG_LATENCY)."""
        flags = abi.CONFIG_PROFILE if profile else 0
        if pipeline is not None:
            flags |= abi.CONFIG_PIPELINE if pipeline else abi.CONFIG_LATENCY
        cfg = abi.Config(device, block_size, arena_bytes, flags, 0)
        h = ctypes.c_void_p()
        check(lib().tbc_engine_init(ctypes.byref(cfg), ctypes.byref(h)), "tbc_engine_init")
        self.handle = h.value
        self.block_size = block_size
        self._prepared = None

    def close(self) -> None:
        if self.handle:
            lib().tbc_engine_deinit(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def layout(self, tree: TreeSpec) -> abi.TreeLayout:
        out = abi.TreeLayout()
        t = tree.ctype()
        check(lib().tbc_tree_layout_get(self.handle, ctypes.byref(t), ctypes.byref(out)), "tbc_tree_layout_get")
        return out

    def arena_usage(self) -> tuple:
        """(device bytes, pinned host bytes, open regions) of the static arenas
        held by unreleased batches and k-way merges (tbc_engine_arena_usage)."""
        d, h, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
        check(lib().tbc_engine_arena_usage(self.handle, ctypes.byref(d), ctypes.byref(h), ctypes.byref(n)),
              "tbc_engine_arena_usage")
        return d.value, h.value, n.value

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def host_register(self, array: np.ndarray) -> None:
        """tbc_host_register: grid block transfers into or out of this
        (contiguous) host array go by DMA without the staging ring's copy.
        The caller keeps the array alive until host_unregister."""
        assert array.flags.c_contiguous and array.nbytes
        check(lib().tbc_host_register(self.handle, array.ctypes.data, array.nbytes), "tbc_host_register")

    def host_unregister(self, array: np.ndarray) -> None:
        check(lib().tbc_host_unregister(self.handle, array.ctypes.data), "tbc_host_unregister")

    def upload(self, array: np.ndarray, pad: int = 0) -> DeviceBuffer:
        a = np.ascontiguousarray(array)
        buf = DeviceBuffer(self, a.nbytes + pad)
        if a.nbytes:
            buf.upload(a)
        return buf

    def synchronize(self) -> None:
        check(lib().tbc_synchronize(self.handle), "tbc_synchronize")

    def checksum(self, messages: list) -> list:
        """vsr.checksum of each message (bytes), computed on the GPU."""
        bufs, ptrs, lens = [], [], []
        for m in messages:
            m = bytes(m)
            b = self.upload(np.frombuffer(m + b"\0" * 4, dtype=np.uint8))
            bufs.append(b)
            ptrs.append(b.ptr)
            lens.append(len(m))
        n = len(messages)
        P = (ctypes.c_void_p * max(1, n))(*ptrs)
        L = (ctypes.c_uint64 * max(1, n))(*lens)
        out = np.zeros(16 * max(1, n), dtype=np.uint8)
        check(lib().tbc_checksum_batch(self.handle, P, L, n, out.ctypes.data), "tbc_checksum_batch")
        return [int.from_bytes(out[16 * i:16 * i + 16].tobytes(), "little") for i in range(n)]

    def checksum_device(self, ptrs: list, lens: list) -> np.ndarray:
        n = len(ptrs)
        P = (ctypes.c_void_p * max(1, n))(*ptrs)
        L = (ctypes.c_uint64 * max(1, n))(*lens)
        out = np.zeros(16 * max(1, n), dtype=np.uint8)
        check(lib().tbc_checksum_batch(self.handle, P, L, n, out.ctypes.data), "tbc_checksum_batch")
        return out[: 16 * n].reshape(n, 16)

    def validate_blocks(self, ptrs: list, expect_checksums: list, expect_addresses: list) -> np.ndarray:
        """grid.read_block_validate on device-resident blocks (tbc_blocks_validate):
        one tbc_block_check code per block (0 = valid)."""
        n = len(ptrs)
        P = (ctypes.c_void_p * max(1, n))(*ptrs)
        C = np.zeros(2 * max(1, n), dtype=np.uint64)
        for i, c in enumerate(expect_checksums):
            C[2 * i], C[2 * i + 1] = c & ((1 << 64) - 1), c >> 64
        A = np.asarray(list(expect_addresses) + [0], dtype=np.uint64)
        out = np.zeros(max(1, n), dtype=np.uint8)
        check(lib().tbc_blocks_validate(self.handle, P, C.ctypes.data, A.ctypes.data, n, out.ctypes.data),
              "tbc_blocks_validate")
        return out[:n]

    def sort_values(self, tree: TreeSpec, buf: DeviceBuffer, count: int, sync: bool = True) -> None:
        t = tree.ctype()
        f = lib().tbc_sort_values if sync else lib().tbc_sort_values_async
        check(f(self.handle, ctypes.byref(t), buf.ptr, count), "tbc_sort_values")

    def copy_device_async(self, dst: int, src: int, nbytes: int) -> None:
        check(lib().tbc_copy_device_async(self.handle, dst, src, nbytes), "tbc_copy_device_async")

    def copy_device_batch(self, copies: list) -> None:
        """tbc_copy_device_batch: [(dst, src, nbytes)] device copies in one
        launch on the engine stream (no host wait)."""
        arr = (abi.Copy * max(1, len(copies)))()
        for i, (d, s, n) in enumerate(copies):
            arr[i].dst, arr[i].src, arr[i].bytes = d, s, n
        check(lib().tbc_copy_device_batch(self.handle, arr, len(copies)), "tbc_copy_device_batch")

    def sort_values_batch(self, tables: list) -> None:
        """Bar end: [(TreeSpec, DeviceBuffer | device ptr, count[, out])] sorted
        by one segmented launch sequence (tbc_sort_values_batch), enqueued on
        the engine stream; with `out` (a device pointer) a table is sorted out
        of place into it and its values are only read."""
        arr = (abi.SortJob * max(1, len(tables)))()
        for i, (tree, buf, n, *out) in enumerate(tables):
            arr[i].tree = tree.ctype()
            arr[i].values = buf if isinstance(buf, int) else buf.ptr
            arr[i].count = n
            arr[i].values_out = out[0] if out else None
        check(lib().tbc_sort_values_batch(self.handle, arr, len(tables)), "tbc_sort_values_batch")

    def kway_merge(self, tree: TreeSpec, streams: list, out: DeviceBuffer, descending: bool = False) -> int:
        """Scan-path k-way merge (tbc_kway_merge; k_way_merge.zig:8-205 with a
        higher stream index winning equal keys): `streams` = [(device ptr,
        count)] sorted in the merge direction; returns the merged count."""
        arr = (abi.Segment * max(1, len(streams)))()
        for i, (p, n) in enumerate(streams):
            arr[i].values, arr[i].count = p, n
        t = tree.ctype()
        n_out = ctypes.c_uint64()
        check(lib().tbc_kway_merge(self.handle, ctypes.byref(t), arr, len(streams), int(descending),
                                   out.ptr if out is not None else None, ctypes.byref(n_out)), "tbc_kway_merge")
        return n_out.value

    def kway_merge_submit(self, tree: TreeSpec, streams: list, out: DeviceBuffer, descending: bool = False):
        """tbc_kway_merge_submit: enqueue the merge and return a KwayMerge
        handle at once (poll() / wait(), then count())."""
        arr = (abi.Segment * max(1, len(streams)))()
        for i, (p, n) in enumerate(streams):
            arr[i].values, arr[i].count = p, n
        t = tree.ctype()
        h = ctypes.c_void_p()
        check(lib().tbc_kway_merge_submit(self.handle, ctypes.byref(t), arr, len(streams), int(descending),
                                          out.ptr if out is not None else None, ctypes.byref(h)),
              "tbc_kway_merge_submit")
        return KwayMerge(h)

    def prepare(self, jobs: list):
        """The tbc_compaction[] array of a job list (cached for a repeated list)."""
        key = tuple(id(j) for j in jobs)
        if self._prepared is not None and self._prepared[0] == key:
            return self._prepared[1]
        arr = (abi.Compaction * max(1, len(jobs)))()
        for i, j in enumerate(jobs):
            arr[i] = j.ctype()
        self._prepared = (key, arr, list(jobs))
        return arr

    def submit(self, jobs: list) -> Batch:
        arr = self.prepare(jobs)
        h = ctypes.c_void_p()
        check(lib().tbc_compaction_submit(self.handle, arr, len(jobs), ctypes.byref(h)), "tbc_compaction_submit")
        return Batch(self, h.value, jobs)

    def set_profile(self, on: bool) -> None:
        """Profile marks (kernel_times) for the batches submitted from now on
        (tbc_engine_set_profile): timed loops run without them."""
        check(lib().tbc_engine_set_profile(self.handle, 1 if on else 0), "tbc_engine_set_profile")

    def stream_handle(self) -> int:
        """The engine stream (tbc_engine_stream), for torch.cuda.ExternalStream."""
        p = ctypes.c_void_p()
        check(lib().tbc_engine_stream(self.handle, ctypes.byref(p)), "tbc_engine_stream")
        return p.value

    def seal(self, tree: TreeSpec, cluster: int, snapshot_min: int, level_b: int, addresses, arena,
             value_count: int, blocks: tuple, tables: tuple):
        """tbc_compaction_seal of one split job (blocking): finish data blocks
        [blocks[0], blocks[1]) in place (headers, checksums, index entries),
        then seal tables [tables[0], tables[1]) from the entries in their index
        block slots. Returns (result, TableInfos of the sealed tables)."""
        b = self.seal_submit(tree, cluster, snapshot_min, level_b, addresses, arena, value_count, blocks, tables)
        try:
            b.wait()
            r, infos = b.result(0)
            check(r.status, "tbc_compaction_seal")
            return r, infos
        finally:
            b.release()

    def seal_submit(self, tree: TreeSpec, cluster: int, snapshot_min: int, level_b: int, addresses, arena,
                    value_count: int, blocks: tuple, tables: tuple) -> Batch:
        """tbc_compaction_seal, enqueued: returns the batch (wait, then
        result(0) for the sealed tables' TableInfos). `arena.ptr` is the
        job's output slot 0 (a rank holding only its own slots passes its
        allocation minus the slots before them)."""
        addrs = np.ascontiguousarray(addresses, dtype=np.uint64)
        sl = abi.Seal()
        sl.tree = tree.ctype()
        sl.cluster[0], sl.cluster[1] = cluster & ((1 << 64) - 1), cluster >> 64
        sl.snapshot_min = snapshot_min
        sl.level_b = level_b
        sl.address_count = len(addrs)
        sl.addresses = addrs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        sl.output_blocks = arena.ptr
        sl.value_count = value_count
        sl.block_first, sl.block_count = blocks[0], blocks[1] - blocks[0]
        sl.table_first, sl.table_count = tables[0], tables[1] - tables[0]
        h = ctypes.c_void_p()
        check(lib().tbc_compaction_seal(self.handle, ctypes.byref(sl), ctypes.byref(h)), "tbc_compaction_seal")
        b = Batch(self, h.value, [None])
        b._keep = addrs  # the host address array outlives the enqueue
        return b


def stage_blocks(engine: Engine, tables: list, value_size: int, block_size: int = BLOCK_SIZE):
    """Place each input data block's values at +256 of its own block in one
    device buffer (the grid's block layout) and return (buffer, segments)."""
    nblocks = sum(len(t) for t in tables)
    host = np.zeros((max(1, nblocks), block_size), dtype=np.uint8)
    segs_host = []
    k = 0
    for table in tables:
        for vals in table:
            v = np.ascontiguousarray(vals, dtype=np.uint8).reshape(-1)
            host[k, HEADER_SIZE:HEADER_SIZE + v.size] = v
            segs_host.append((k, v.size // value_size))
            k += 1
    buf = engine.upload(host)
    segs = [(buf.ptr + i * block_size + HEADER_SIZE, n) for i, n in segs_host]
    return buf, segs
