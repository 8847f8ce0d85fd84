"""ctypes wrapper over the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: the parity checker and the CPU baseline. Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module. The product path (tigerbeetle_amd / libtbc.so) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

KEY_TIMESTAMP, KEY_ID_U128, KEY_COMPOSITE_U64, KEY_COMPOSITE_U128 = 0, 1, 2, 3
USAGE_GENERAL, USAGE_SECONDARY_INDEX = 0, 1


def build() -> str:
    """Compile the oracle in-tree (make)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


class Tree(ctypes.Structure):
    _fields_ = [
        ("tree_id", ctypes.c_uint16),
        ("key_kind", ctypes.c_uint8),
        ("usage", ctypes.c_uint8),
        ("value_size", ctypes.c_uint32),
        ("timestamp_offset", ctypes.c_uint32),
        ("key_size", ctypes.c_uint32),
        ("block_size", ctypes.c_uint32),
        ("block_value_count_max", ctypes.c_uint32),
        ("data_block_count_max", ctypes.c_uint32),
        ("value_count_max", ctypes.c_uint32),
        ("index_size", ctypes.c_uint32),
        ("index_checksums_offset", ctypes.c_uint32),
        ("index_keys_min_offset", ctypes.c_uint32),
        ("index_keys_max_offset", ctypes.c_uint32),
        ("index_addresses_offset", ctypes.c_uint32),
    ]


class Segment(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("count", ctypes.c_uint32)]


class Job(ctypes.Structure):
    _fields_ = [
        ("tree", ctypes.POINTER(Tree)),
        ("a_immutable", ctypes.c_int),
        ("segments_a", ctypes.POINTER(Segment)),
        ("segment_count_a", ctypes.c_uint32),
        ("segments_b", ctypes.POINTER(Segment)),
        ("segment_count_b", ctypes.c_uint32),
        ("drop_tombstones", ctypes.c_int),
        ("level_b", ctypes.c_uint8),
        ("cluster_lo", ctypes.c_uint64),
        ("cluster_hi", ctypes.c_uint64),
        ("snapshot_min", ctypes.c_uint64),
        ("addresses", ctypes.POINTER(ctypes.c_uint64)),
        ("address_count", ctypes.c_uint32),
        ("out_blocks", ctypes.c_void_p),
        ("out_block_capacity", ctypes.c_uint32),
        ("out_table_infos", ctypes.c_void_p),
        ("out_table_capacity", ctypes.c_uint32),
        ("out_value_count", ctypes.c_uint64),
        ("out_data_block_count", ctypes.c_uint32),
        ("out_table_count", ctypes.c_uint32),
        ("out_block_count", ctypes.c_uint32),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.tbo_checksum.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        _lib.tbo_checksum.restype = None
        _lib.tbo_has_aesni.restype = ctypes.c_int
        _lib.tbo_force_portable.argtypes = [ctypes.c_int]
        _lib.tbo_aegis_seed_state.argtypes = [ctypes.c_void_p]
        _lib.tbo_tree_init.argtypes = [ctypes.POINTER(Tree), ctypes.c_uint16, ctypes.c_uint8,
                                       ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint32]
        _lib.tbo_tree_init.restype = ctypes.c_int
        _lib.tbo_sort_values.argtypes = [ctypes.POINTER(Tree), ctypes.c_void_p, ctypes.c_uint32]
        _lib.tbo_sort_values.restype = ctypes.c_int
        _lib.tbo_compact.argtypes = [ctypes.POINTER(Job)]
        _lib.tbo_compact.restype = ctypes.c_int
        _lib.tbo_key.argtypes = [ctypes.POINTER(Tree), ctypes.c_void_p, ctypes.c_void_p]
        _lib.tbo_tombstone.argtypes = [ctypes.POINTER(Tree), ctypes.c_void_p]
        _lib.tbo_tombstone_from_key.argtypes = [ctypes.POINTER(Tree), ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def checksum(data: bytes | np.ndarray, portable: bool = False) -> int:
    """vsr.checksum (src/vsr/checksum.zig:50) as a Python int (u128)."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = (ctypes.c_uint8 * 16)()
    lib().tbo_force_portable(1 if portable else 0)
    try:
        lib().tbo_checksum(buf.ctypes.data if buf.size else None, buf.size, out)
    finally:
        lib().tbo_force_portable(0)
    return int.from_bytes(bytes(out), "little")


def seed_state() -> bytes:
    out = (ctypes.c_uint8 * 128)()
    lib().tbo_aegis_seed_state(out)
    return bytes(out)


def tree(tree_id, key_kind, usage, value_size, timestamp_offset, table_value_count_max,
         block_size) -> Tree:
    t = Tree()
    rc = lib().tbo_tree_init(ctypes.byref(t), tree_id, key_kind, usage, value_size,
                             timestamp_offset, table_value_count_max, block_size)
    if rc != 0:
        raise ValueError(f"tbo_tree_init failed: {rc}")
    return t


def sort_values(t: Tree, values: np.ndarray) -> np.ndarray:
    """TableMemory.sort: stable sort by key; returns a sorted copy (rows = values)."""
    v = np.ascontiguousarray(values, dtype=np.uint8).copy()
    n = v.shape[0]
    rc = lib().tbo_sort_values(ctypes.byref(t), v.ctypes.data, n)
    if rc != 0:
        raise RuntimeError(f"tbo_sort_values failed: {rc}")
    return v


class CompactionResult:
    def __init__(self, status, blocks, table_infos, value_count, data_block_count):
        self.status = status
        self.blocks = blocks  # (block_count, block_size) uint8, acquire order
        self.table_infos = table_infos  # (table_count, 128) uint8
        self.value_count = value_count
        self.data_block_count = data_block_count


def compact(t: Tree, a_segments, b_segments, *, a_immutable: bool, drop_tombstones: bool,
            level_b: int, cluster: int, snapshot_min: int, addresses) -> CompactionResult:
    """One Compaction (A = immutable sorted table or disk-table blocks, B =
    level-B blocks). Segments are 2-D uint8 arrays, one row per value."""
    keep = []

    def segs(lst):
        arr = (Segment * max(1, len(lst)))()
        for i, s in enumerate(lst):
            s = np.ascontiguousarray(s, dtype=np.uint8)
            keep.append(s)
            arr[i].values = s.ctypes.data if s.size else None
            arr[i].count = s.shape[0]
        return arr

    sa, sb = segs(a_segments), segs(b_segments)
    addrs = np.ascontiguousarray(np.asarray(addresses, dtype=np.uint64))
    cap = len(addrs)
    out_blocks = np.zeros((max(cap, 1), t.block_size), dtype=np.uint8)
    tables_cap = cap
    out_infos = np.zeros((max(tables_cap, 1), 128), dtype=np.uint8)
    job = Job()
    job.tree = ctypes.pointer(t)
    job.a_immutable = int(a_immutable)
    job.segments_a = sa
    job.segment_count_a = len(a_segments)
    job.segments_b = sb
    job.segment_count_b = len(b_segments)
    job.drop_tombstones = int(drop_tombstones)
    job.level_b = level_b
    job.cluster_lo = cluster & ((1 << 64) - 1)
    job.cluster_hi = cluster >> 64
    job.snapshot_min = snapshot_min
    job.addresses = addrs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    job.address_count = cap
    job.out_blocks = out_blocks.ctypes.data
    job.out_block_capacity = cap
    job.out_table_infos = out_infos.ctypes.data
    job.out_table_capacity = tables_cap
    rc = lib().tbo_compact(ctypes.byref(job))
    return CompactionResult(rc, out_blocks[: job.out_block_count],
                            out_infos[: job.out_table_count], job.out_value_count,
                            job.out_data_block_count)


def kway_merge(streams: list, descending: bool = False) -> list:
    """KWayMergeIteratorType (src/lsm/k_way_merge.zig:8-205), restated line by
    line as a binary heap over stream heads, with the reference tests'
    stream_precedence(a, b) = a > b (:239-244). `streams` are lists of
    (key, payload), each sorted in the merge direction; returns the popped
    (key, payload) list. Pure Python: small inputs (test checker only)."""
    streams = [list(s) for s in streams]
    pos = [0] * len(streams)
    keys, ids = [None] * len(streams), [0] * len(streams)
    k = 0

    def peek(s):  # stream_peek: None = error.Empty (no Drained: all data resident)
        return streams[s][pos[s]][0] if pos[s] < len(streams[s]) else None

    def ordered(a, b):  # :197-203
        if b is None:
            return True
        ka, kb = keys[a], keys[b]
        if ka == kb:
            return ids[a] > ids[b]
        return (ka < kb) != descending

    def swap(a, b):
        keys[a], keys[b] = keys[b], keys[a]
        ids[a], ids[b] = ids[b], ids[a]

    def up_heap(i):  # :134-140
        while i > 0:
            p = (i - 1) // 2
            if ordered(p, i):
                break
            swap(p, i)
            i = p

    def down_heap():  # :145-175
        if k == 0:
            return
        i = 0
        for _ in range(k.bit_length()):
            left = 2 * i + 1 if 2 * i + 1 < k else None
            right = 2 * i + 2 if 2 * i + 2 < k else None
            if ordered(i, left):
                if ordered(i, right):
                    break
                swap(i, right)
                i = right
            elif ordered(i, right):
                swap(i, left)
                i = left
            elif ordered(left, right):
                swap(i, left)
                i = left
            else:
                swap(i, right)
                i = right

    for s in range(len(streams)):  # init, :71-82
        key = peek(s)
        if key is None:
            continue
        keys[k], ids[k] = key, s
        up_heap(k)
        k += 1

    out, previous = [], None
    while True:
        # pop_internal, :109-132: re-key the root from its stream's current
        # head (the value popped last time came from it), then pop the root.
        if k == 0:
            break
        s0 = ids[0]
        key = peek(s0)
        if key is not None:
            keys[0] = key
            down_heap()
        else:
            swap(0, k - 1)
            k -= 1
            down_heap()
        if k == 0:
            break
        root = ids[0]
        value = streams[root][pos[root]]
        pos[root] += 1
        # pop, :91-107
        if previous is not None and value[0] == previous:
            continue
        previous = value[0]
        out.append(value)
    return out


def manifest_blocks(table_infos: np.ndarray, addresses, cluster: int, block_size: int,
                    previous_checksum: int = 0, previous_address: int = 0):
    """ManifestLog.acquire_block/append/close_block (src/lsm/manifest_log.zig:
    876-952) with schema.ManifestNode (src/lsm/schema.zig:451-595), restated
    on the CPU with this oracle's KAT-pinned vsr.checksum. Returns (disk
    images [0, sector_ceil(size)), header checksums)."""
    infos = np.ascontiguousarray(table_infos, dtype=np.uint8).reshape(-1, 128)
    entry_max = (block_size - 256) // 128                      # schema.zig:454
    out, sums = [], []
    prev_c, prev_a = int(previous_checksum), int(previous_address)
    for b, start in enumerate(range(0, len(infos), entry_max)):
        chunk = infos[start:start + entry_max]
        size = 256 + 128 * len(chunk)                          # ManifestNode.size, :574-580
        blk = bytearray(-(-size // 4096) * 4096)
        blk[80:96] = int(cluster).to_bytes(16, "little")       # header.cluster (:893)
        blk[96:100] = size.to_bytes(4, "little")               # header.size (:921)
        blk[110] = 20                                          # command = .block
        blk[128:144] = prev_c.to_bytes(16, "little")           # Metadata (:925-929, schema.zig:475-486)
        blk[160:168] = prev_a.to_bytes(8, "little")
        blk[168:172] = len(chunk).to_bytes(4, "little")
        blk[224:232] = int(addresses[b]).to_bytes(8, "little")  # header.address (:889,894)
        blk[240] = 3                                           # block_type = .manifest
        blk[256:size] = chunk.tobytes()
        blk[32:48] = checksum(bytes(blk[256:size])).to_bytes(16, "little")   # set_checksum_body (:934)
        c = checksum(bytes(blk[16:256]))                       # set_checksum (:935)
        blk[0:16] = c.to_bytes(16, "little")
        out.append(np.frombuffer(bytes(blk), np.uint8))
        sums.append(c)
        prev_c, prev_a = c, int(addresses[b])                  # log_block_checksums/addresses push (:938-939)
    return out, sums
