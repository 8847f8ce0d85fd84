"""The manifest log: events, blocks and compaction.

The reference records every change a compaction makes to a tree's Manifest
as a 128-byte `ManifestNode.TableInfo` entry whose label says insert, update
or remove (schema.zig:489-530):

  Compaction.apply_to_manifest (compaction.zig:939-973): an update per input
    table (snapshot_max := op_min + half - 1; disk A at level_b - 1, every B
    table at level_b), then an insert per output table at level_b — or, for a
    move, one update of the moved table at level_b (Manifest.move_table,
    manifest.zig:283-320: no remove from level_a);
  Manifest.remove_invisible_tables (manifest.zig:345-386), from
    Tree.compact_end (tree.zig:905-953): a remove per input table, now
    invisible, in the level's descending (key_max, snapshot_min) order.

`ManifestLog` (manifest_log.zig) appends the entries to its open block,
closes a block when it holds `entry_count_max = (block_size - 256) / 128`
entries (close_block, :876-952: header with the previous block's checksum
and address, checksum_body, checksum), writes closed blocks at the next
flush, and at every half-bar start compacts the oldest blocks (compact,
:571-809): entries that are still a table's latest extent are re-appended,
the rest dropped, the block released; the number of blocks per half-bar is
paced (Pace, :1077-1239). Its blocks come from its own grid reservation,
made after the trees' reservations (Forest.compact, forest.zig:319-342).

The log's state machine is host logic in the reference and stays host logic
here (this module restates it, as forest.py restates the Forest schedule).
Block closing is the data-parallel part: `GridManifestStore` packs the block
images on the host and closes them on the GPU inside the grid
(tbc_manifest_close_blocks: body checksums in parallel, then the header
chain on one wave, each header linking the previous block's checksum read
from the grid — no host wait). Tests close the same blocks with the oracle
(tests/oracle_executor.py) and compare every block byte for byte.
"""
from __future__ import annotations

import ctypes
from collections import deque

import numpy as np

from . import abi
from .tables import EVENT_INSERT, EVENT_REMOVE, EVENT_UPDATE
from .trees import HEADER_SIZE, LSM_BATCH_MULTIPLE, LSM_GROWTH_FACTOR, LSM_LEVELS, SECTOR_SIZE

TABLE_INFO_SIZE = 128
BLOCK_TYPE_MANIFEST = 3   # schema.zig:57-65
COMMAND_BLOCK = 20        # vsr.zig:196
TREE_COUNT = 21           # state_machine.zig:78-111 tree ids 1..21 (forest_tree_count)
COMPACT_EXTRA_BLOCKS = 1  # config.zig:144 lsm_manifest_compact_extra_blocks (production)
COMPACTIONS_MAX = -(-LSM_LEVELS // 2)                 # tree.zig:77
TABLES_INPUT_MAX = 1 + LSM_GROWTH_FACTOR              # tree.zig:70
TABLES_OUTPUT_MAX = TABLES_INPUT_MAX                  # tree.zig:74
# tree.zig:59-62 table_count_max_for_tree(growth, levels), passed as the
# forest's table count max (forest.zig:199-204).
TABLE_COUNT_MAX = sum(LSM_GROWTH_FACTOR ** (lvl + 1) for lvl in range(LSM_LEVELS))


def entry_count_max(block_size: int) -> int:
    """schema.ManifestNode.entry_count_max (schema.zig:452)."""
    return (block_size - HEADER_SIZE) // TABLE_INFO_SIZE


def pack_blocks(table_infos: np.ndarray, addresses, cluster: int, block_size: int,
                previous_address: int = 0) -> list:
    """Headers (checksums and previous-checksum links still zero) and bodies of
    the manifest blocks holding `table_infos` in order, one per address
    (ManifestLog.acquire_block :858-874 and close_block :896-912)."""
    infos = np.ascontiguousarray(table_infos, dtype=np.uint8).reshape(-1, TABLE_INFO_SIZE)
    m = entry_count_max(block_size)
    blocks = []
    for b, start in enumerate(range(0, len(infos), m)):
        chunk = infos[start:start + m]
        size = HEADER_SIZE + len(chunk) * TABLE_INFO_SIZE
        blk = np.zeros(-(-size // SECTOR_SIZE) * SECTOR_SIZE, dtype=np.uint8)  # zero padding (:931-932)
        h = blk[:HEADER_SIZE]
        h[80:96] = np.frombuffer(int(cluster).to_bytes(16, "little"), np.uint8)
        h[96:100] = np.frombuffer(np.uint32(size).tobytes(), np.uint8)
        h[110] = COMMAND_BLOCK
        prev_addr = previous_address if b == 0 else int(addresses[b - 1])
        h[160:168] = np.frombuffer(np.uint64(prev_addr).tobytes(), np.uint8)
        h[168:172] = np.frombuffer(np.uint32(len(chunk)).tobytes(), np.uint8)
        h[224:232] = np.frombuffer(np.uint64(int(addresses[b])).tobytes(), np.uint8)
        h[240] = BLOCK_TYPE_MANIFEST
        blk[HEADER_SIZE:size] = chunk.reshape(-1)
        blocks.append(blk)
    return blocks


def close_on_grid(grid, images: list, addresses, previous_address: int = 0, previous_checksum: int | None = None):
    """tbc_manifest_close_blocks: stage packed images into the grid and close
    them on the device (enqueued; no host wait)."""
    n = len(images)
    if n == 0:
        return
    A = np.ascontiguousarray(np.asarray(addresses, dtype=np.uint64))
    keep = [np.ascontiguousarray(im) for im in images]
    P = (ctypes.c_void_p * n)(*[im.ctypes.data for im in keep])
    prev = None
    if previous_checksum is not None:
        prev = np.array([previous_checksum & ((1 << 64) - 1), previous_checksum >> 64], dtype=np.uint64)
    abi.check(abi.lib().tbc_manifest_close_blocks(
        grid.handle, A.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), P, n, int(previous_address),
        prev.ctypes.data if prev is not None else None), "tbc_manifest_close_blocks")


def manifest_blocks(grid, table_infos: np.ndarray, addresses, cluster: int, previous_checksum: int = 0,
                    previous_address: int = 0):
    """Close the manifest blocks of `table_infos` (one per address) on the GPU
    into `grid`, then read them back: (disk images, header checksums)."""
    bs = grid.engine.block_size
    images = pack_blocks(table_infos, addresses, cluster, bs, previous_address)
    if not images:
        return [], []
    if len(addresses) < len(images):
        raise ValueError("one address per manifest block")
    close_on_grid(grid, images, list(addresses)[:len(images)], previous_address, previous_checksum)
    got = grid.get_blocks(list(addresses)[:len(images)])
    out = [g[:len(im)].copy() for g, im in zip(got, images)]
    return out, [int.from_bytes(g[0:16].tobytes(), "little") for g in out]


class Pace:
    """ManifestLog.Pace (manifest_log.zig:1077-1239)."""

    def __init__(self, tree_count: int, tables_max: int, compact_extra_blocks: int, block_entries_max: int):
        assert tree_count > 0 and tables_max > tree_count and compact_extra_blocks > 0
        append_entries = tree_count * COMPACTIONS_MAX * (TABLES_INPUT_MAX + TABLES_INPUT_MAX + TABLES_OUTPUT_MAX)
        self.half_bar_append_blocks_max = -(-append_entries // block_entries_max)            # "A"
        self.half_bar_compact_blocks_max = self.half_bar_append_blocks_max + compact_extra_blocks  # "C"
        self.log_blocks_full_max = -(-tables_max // block_entries_max)                     # "T"
        before = 0
        for _ in range(1024):
            after = self.log_blocks_full_max + self.half_bar_append_blocks_max * \
                -(-before // self.half_bar_compact_blocks_max)
            if after == before:
                break
            before = after
        else:
            raise AssertionError("ManifestLog.Pace.log_blocks_cycle_max: no convergence")
        self.log_blocks_cycle_max = after
        burst = self.half_bar_append_blocks_max * -(-(self.log_blocks_full_max + 1) // self.half_bar_compact_blocks_max)
        self.log_blocks_max = self.log_blocks_cycle_max + burst
        self.tables_max = tables_max
        assert self.log_blocks_cycle_max > self.log_blocks_full_max

    def half_bar_compact_blocks(self, log_blocks_count: int, tables_count: int) -> int:
        assert tables_count <= self.tables_max
        if self.log_blocks_cycle_max <= log_blocks_count + self.half_bar_append_blocks_max:
            return self.half_bar_compact_blocks_max
        target = max(1, self.log_blocks_cycle_max * tables_count // self.tables_max)
        return min(self.half_bar_compact_blocks_max, self.half_bar_compact_blocks_max * log_blocks_count // target)


class ManifestLog:
    """ManifestLogType (manifest_log.zig) after open() on an empty log.

    `store` closes and reads blocks: close(infos (n, 128), address,
    previous_address) and read(address) -> block image (GridManifestStore on
    the GPU grid; the oracle's store in tests). `free_set` is the forest's
    (forest.FreeSet): the log reserves its blocks after the trees do."""

    def __init__(self, store, free_set, block_size: int, tree_count: int = TREE_COUNT,
                 tables_max: int = TABLE_COUNT_MAX, compact_extra_blocks: int = COMPACT_EXTRA_BLOCKS):
        self.store, self.free_set = store, free_set
        self.entry_count_max = entry_count_max(block_size)
        self.pace = Pace(tree_count, tables_max, compact_extra_blocks, self.entry_count_max)
        # log_block_checksums / log_block_addresses (oldest first): closed
        # blocks, written or not. Checksums are the store's to know.
        self.log_addresses: deque = deque()
        self.open_entries: list = []       # the open block's entries (entry_count of them)
        self.open_address = 0
        self.blocks_closed = 0             # closed and not yet flushed
        self.table_extents: dict = {}      # table address -> (manifest block address, entry)
        self.reservation = None
        self.compact_blocks = None
        self.stats = {"appends": 0, "blocks_closed": 0, "blocks_compacted": 0, "entries_dropped": 0}

    @property
    def entry_count(self) -> int:
        return len(self.open_entries)

    # -- append ----------------------------------------------------------
    def append(self, entry: np.ndarray) -> None:
        """ManifestLog.append (:451-468): an external event."""
        address = int(entry[96:104].view(np.uint64)[0])
        event = int(entry[126]) >> 6
        if event == EVENT_INSERT:
            assert address not in self.table_extents
        else:
            assert event in (EVENT_UPDATE, EVENT_REMOVE) and address in self.table_extents
        self.append_internal(entry)

    def append_internal(self, entry: np.ndarray) -> None:
        """:476-535: into the open block (acquired on the first entry), the
        table's extent updated at once; a full block is closed."""
        assert self.reservation is not None, "appends happen inside a half-bar with the log's reservation"
        e = np.ascontiguousarray(entry, dtype=np.uint8).reshape(TABLE_INFO_SIZE)
        level, event = int(e[126]) & 0x3f, int(e[126]) >> 6
        address = int(e[96:104].view(np.uint64)[0])
        smin, smax = (int(x) for x in e[104:120].view(np.uint64))
        assert level < LSM_LEVELS and address > 0 and smin > 0 and smax > smin
        if not self.open_entries:
            self.acquire_block()
        index = len(self.open_entries)
        self.open_entries.append(e.copy())
        if event in (EVENT_INSERT, EVENT_UPDATE):
            self.table_extents[address] = (self.open_address, index)
        else:
            assert event == EVENT_REMOVE
            del self.table_extents[address]
        self.stats["appends"] += 1
        if len(self.open_entries) == self.entry_count_max:
            self.close_block()

    def acquire_block(self) -> None:
        """:843-874: the next block address from the log's reservation."""
        self.open_address = self.free_set.acquire_from(self.reservation)

    def close_block(self) -> None:
        """:876-952: header (previous block = the log's newest), checksums —
        done by the store, on the device for the GPU grid."""
        assert self.open_entries
        prev = self.log_addresses[-1] if self.log_addresses else 0
        self.store.close(np.stack(self.open_entries), self.open_address, prev)
        self.log_addresses.append(self.open_address)
        self.blocks_closed += 1
        self.open_entries = []
        self.open_address = 0
        self.stats["blocks_closed"] += 1

    # -- half-bar --------------------------------------------------------
    def flush(self) -> None:
        """:537-640: write the closed blocks. The stores close blocks straight
        into the grid, so a flush only retires them from the buffer."""
        self.blocks_closed = 0

    def compact(self, op: int, skipped: bool = False) -> None:
        """:571-614 then compact_next_block / compact_read_block_callback
        (:628-718): at a half-bar start, after the trees' reservations.
        `skipped`: an op the recovered checkpoint already compacted
        (op_compacted, :659-665)."""
        assert self.reservation is None and self.compact_blocks is None
        assert op % (LSM_BATCH_MULTIPLE // 2) == 0
        if op < LSM_BATCH_MULTIPLE or skipped:
            return
        compact_blocks = min(self.pace.half_bar_compact_blocks(len(self.log_addresses), len(self.table_extents)),
                             len(self.log_addresses) - self.blocks_closed)
        assert compact_blocks <= self.pace.half_bar_compact_blocks_max
        self.reservation = self.free_set.reserve(compact_blocks + self.pace.half_bar_append_blocks_max)
        self.flush()
        for _ in range(compact_blocks):
            oldest = self.log_addresses.popleft()
            block = self.store.read(oldest)
            verify_block(block, oldest)
            n = int(block[168:172].view(np.uint32)[0])
            entries = block[HEADER_SIZE:HEADER_SIZE + n * TABLE_INFO_SIZE].reshape(n, TABLE_INFO_SIZE)
            for k, e in enumerate(entries):
                event = int(e[126]) >> 6
                address = int(e[96:104].view(np.uint64)[0])
                if event in (EVENT_INSERT, EVENT_UPDATE) and self.table_extents.get(address) == (oldest, k):
                    self.append_internal(e)
                else:
                    self.stats["entries_dropped"] += 1
            self.free_set.release(oldest)
            self.stats["blocks_compacted"] += 1
        self.compact_blocks = 0

    def compact_end(self) -> None:
        """:748-765."""
        if self.reservation is not None:
            self.free_set.forfeit()
            self.reservation = None
        else:
            assert not self.open_entries and self.blocks_closed == 0
        self.compact_blocks = None

    def checkpoint(self) -> None:
        """:767-781: close the partial block, flush."""
        assert self.reservation is None or self.compact_blocks is not None
        if self.open_entries:
            self.close_block()
        self.flush()

    def snapshot(self) -> dict:
        """The log's state a checkpoint persists (checkpoint_references plus
        the table extents open() rebuilds, :783-809)."""
        assert not self.open_entries and self.reservation is None
        newest = self.log_addresses[-1] if self.log_addresses else 0
        return {"log_addresses": list(self.log_addresses), "table_extents": dict(self.table_extents),
                "newest": (newest, self.store.checksum(newest) if newest and hasattr(self.store, "checksum") else 0)}

    def restore(self, snap: dict) -> None:
        """ManifestLog.open from the checkpoint's references: the log's
        blocks and the table extents (the blocks themselves stay in the grid)."""
        self.log_addresses = deque(snap["log_addresses"])
        self.table_extents = dict(snap["table_extents"])
        newest, checksum = snap["newest"]
        if newest and hasattr(self.store, "restore_link"):
            self.store.restore_link(newest, checksum)
        self.open_entries, self.open_address, self.blocks_closed = [], 0, 0
        self.reservation, self.compact_blocks = None, None

    def references(self) -> tuple:
        """(oldest address, newest address, block count) of the log
        (checkpoint_references, :783-809; checksums are in the blocks)."""
        if not self.log_addresses:
            return (0, 0, 0)
        return (self.log_addresses[0], self.log_addresses[-1], len(self.log_addresses))


def verify_block(block: np.ndarray, address: int | None = None) -> None:
    """ManifestLog.verify_block's structural asserts (:954-970,
    ManifestNode.metadata schema.zig:534-554)."""
    size = int(block[96:100].view(np.uint32)[0])
    n = int(block[168:172].view(np.uint32)[0])
    assert block[240] == BLOCK_TYPE_MANIFEST and block[110] == COMMAND_BLOCK
    assert address is None or int(block[224:232].view(np.uint64)[0]) == address
    assert n > 0 and n == (size - HEADER_SIZE) // TABLE_INFO_SIZE and (size - HEADER_SIZE) % TABLE_INFO_SIZE == 0
    assert not block[144:160].any() and not block[172:224].any()


def open_log(blocks_oldest_first: list) -> dict:
    """ManifestLog.open (:266-403, strategy 2 of Forest.verify_tables_recovered,
    forest.zig:560-650): newest block first, entries in reverse, removes
    remembered until their insert, the first (latest) insert/update of every
    other table kept. Returns {table address: entry}."""
    removed, latest = set(), {}
    for block in reversed(blocks_oldest_first):
        n = int(block[168:172].view(np.uint32)[0])
        entries = block[HEADER_SIZE:HEADER_SIZE + n * TABLE_INFO_SIZE].reshape(n, TABLE_INFO_SIZE)
        for e in entries[::-1]:
            event = int(e[126]) >> 6
            address = int(e[96:104].view(np.uint64)[0])
            if event == EVENT_REMOVE:
                assert address not in removed
                removed.add(address)
            elif address in removed:
                if event == EVENT_INSERT:
                    removed.discard(address)
            elif address not in latest:
                latest[address] = e.copy()
    return latest


def replay_log(blocks_oldest_first: list) -> dict:
    """Strategy 1 of Forest.verify_tables_recovered (forest.zig:587-620):
    every event in chronological order, keyed by table checksum."""
    tables: dict = {}
    for block in blocks_oldest_first:
        n = int(block[168:172].view(np.uint32)[0])
        for e in block[HEADER_SIZE:HEADER_SIZE + n * TABLE_INFO_SIZE].reshape(n, TABLE_INFO_SIZE):
            checksum = int.from_bytes(e[64:80].tobytes(), "little")
            if int(e[126]) >> 6 == EVENT_REMOVE:
                tables.pop(checksum, None)
            else:
                tables[checksum] = e.copy()
    return tables


class GridManifestStore:
    """Manifest blocks closed on the GPU into the grid (tbc_manifest_close_blocks)
    and read back from it (tbc_grid_get_blocks) when the log compacts them."""

    def __init__(self, grid, cluster: int, record: list | None = None):
        self.grid, self.cluster = grid, cluster
        self.block_size = grid.engine.block_size
        self.record = record
        self.closed: list = []
        self.links: dict = {}  # address -> header checksum the host knows (a recovered log's newest block)

    def checksum(self, address: int) -> int:
        """A closed block's header checksum (what the checkpoint's
        references record for the log's newest block, manifest_log.zig:783-809).
        Raises if a close of this grid was refused (tbc_manifest_close_status)."""
        self.grid.manifest_close_status()
        blk = self.grid.get_blocks([address])[0]
        return int.from_bytes(blk[:16].tobytes(), "little")

    def restore_link(self, address: int, checksum: int) -> None:
        """After a restart the grid's cache is cold: the next block links the
        newest block by the checksum recovered with the log, not by reading a
        trusted grid block."""
        self.links[int(address)] = int(checksum)

    def close(self, infos: np.ndarray, address: int, previous_address: int) -> None:
        images = pack_blocks(infos, [address], self.cluster, self.block_size, previous_address)
        assert len(images) == 1
        prev = self.links.pop(int(previous_address), None) if previous_address else 0
        close_on_grid(self.grid, images, [address], previous_address, prev)
        if self.record is not None:
            self.record.append(("manifest", images, [address], previous_address))
        self.closed.append(address)

    def read(self, address: int) -> np.ndarray:
        blk = self.grid.get_blocks([address])[0]
        size = int(blk[96:100].view(np.uint32)[0])
        return blk[:-(-size // SECTOR_SIZE) * SECTOR_SIZE].copy()
