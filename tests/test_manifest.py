"""Manifest-log blocks: the oracle restatement of
ManifestLog.close_block (manifest_log.zig:876-952) checked against the
reference's structural asserts (schema.zig:534-554 ManifestNode.metadata,
:574-580 size, manifest_log.zig:954-960 verify_block) and the chain links;
the GPU path (tigerbeetle_amd/manifest.py) must equal it byte for byte."""
import numpy as np
import pytest

from oracle import oracle
from tigerbeetle_amd import manifest

CLUSTER = 0xA1B2C3D4E5F60718293A4B5C6D7E8F90


def _infos(n, seed=0):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(n, 128), dtype=np.uint8)


@pytest.mark.parametrize("bs,n", [(4096, 1), (4096, 30), (4096, 31), (4096, 95), (1 << 20, 8190), (1 << 20, 9000)])
def test_oracle_manifest_blocks_structure(bs, n):
    addrs = list(range(500, 600, 7))
    imgs, sums = oracle.manifest_blocks(_infos(n), addrs, CLUSTER, bs, previous_checksum=0x55, previous_address=9)
    m = (bs - 256) // 128
    assert len(imgs) == -(-n // m)
    for b, (img, c) in enumerate(zip(imgs, sums)):
        size = int(img[96:100].view(np.uint32)[0])
        count = int(img[168:172].view(np.uint32)[0])
        assert 0 < count <= m and count == (size - 256) // 128            # schema.zig:542-545
        assert not img[144:160].any() and not img[172:224].any()          # padding, reserved (:546-547)
        assert int(img[232:240].view(np.uint64)[0]) == 0 and img[240] == 3 and img[110] == 20
        assert int(img[224:232].view(np.uint64)[0]) == addrs[b]
        prev_a = int(img[160:168].view(np.uint64)[0])
        prev_c = int.from_bytes(img[128:144].tobytes(), "little")
        assert (prev_a, prev_c) == ((9, 0x55) if b == 0 else (addrs[b - 1], sums[b - 1]))
        assert not img[size:].any()                                        # zero padding (:931-932)
        assert oracle.checksum(img[256:size].tobytes()) == int.from_bytes(img[32:48].tobytes(), "little")
        assert oracle.checksum(img[16:256].tobytes()) == c == int.from_bytes(img[0:16].tobytes(), "little")
        assert np.array_equal(img[256:size].reshape(-1, 128), _infos(n)[b * m:b * m + count])


def test_pack_matches_oracle_layout():
    # host packing of the product path = the oracle's bytes before checksums
    infos = _infos(70, 3)
    imgs, _ = oracle.manifest_blocks(infos, [11, 12, 13], CLUSTER, 4096, previous_address=4)
    packed = manifest.pack_blocks(infos, [11, 12, 13], CLUSTER, 4096, previous_address=4)
    assert len(packed) == len(imgs)
    for p, o in zip(packed, imgs):
        q = o.copy()
        q[0:16] = 0
        q[32:48] = 0
        q[128:144] = 0
        assert np.array_equal(p, q)


@pytest.mark.gpu
@pytest.mark.parametrize("bs,n", [(4096, 1), (4096, 95), (1 << 20, 1000), (1 << 20, 20000)])
def test_gpu_manifest_blocks_equal_oracle(bs, n):
    """tbc_manifest_close_blocks: several blocks closed in one call (bodies in
    parallel, the header chain in order), the first linking a given checksum."""
    from tigerbeetle_amd import Engine, Grid
    addrs = list(range(3, 13))
    with Engine(device=0, block_size=bs) as eng:
        grid = Grid(eng, 16)
        try:
            got, gsums = manifest.manifest_blocks(grid, _infos(n, n), addrs, CLUSTER, previous_checksum=7,
                                                  previous_address=2)
        finally:
            grid.close()
    want, wsums = oracle.manifest_blocks(_infos(n, n), addrs, CLUSTER, bs, previous_checksum=7, previous_address=2)
    assert gsums == wsums
    assert all(np.array_equal(g, w) for g, w in zip(got, want)) and len(got) == len(want)


@pytest.mark.gpu
def test_gpu_manifest_chain_links_a_block_closed_earlier():
    """A close whose first block links the previous block by address only: the
    engine reads that block's header checksum from the grid (no host wait)."""
    from tigerbeetle_amd import Engine, Grid
    bs = 4096
    with Engine(device=0, block_size=bs) as eng:
        grid = Grid(eng, 16)
        try:
            first, sums1 = manifest.manifest_blocks(grid, _infos(40, 1), [5, 6], CLUSTER)
            images = manifest.pack_blocks(_infos(31, 2), [9, 10], CLUSTER, bs, previous_address=6)
            manifest.close_on_grid(grid, images, [9, 10], previous_address=6, previous_checksum=None)
            got = grid.get_blocks([9, 10])
        finally:
            grid.close()
    want, _ = oracle.manifest_blocks(_infos(31, 2), [9, 10], CLUSTER, bs, previous_checksum=sums1[-1],
                                     previous_address=6)
    for g, w in zip(got, want):
        assert np.array_equal(g[:len(w)], w)


@pytest.mark.gpu
def test_gpu_manifest_refuses_to_link_an_untrusted_block():
    """linking by address needs a verified manifest block there.
    A previous address holding a block staged from storage (unverified) or a
    non-manifest block leaves the new blocks unlinked with a zero header
    checksum, so validating them fails; a trusted one links as the oracle."""
    from tigerbeetle_amd import Engine, Grid, abi
    bs = 4096
    with Engine(device=0, block_size=bs) as eng:
        grid = Grid(eng, 16)
        try:
            first, _ = manifest.manifest_blocks(grid, _infos(40, 1), [5, 6], CLUSTER)
            grid.put_blocks([3], np.pad(first[1], (0, bs - len(first[1])))[None])  # a valid manifest image
            for prev in (3, 7):  # 3: staged from storage (unverified); 7: never written (not a manifest block)
                images = manifest.pack_blocks(_infos(31, 2), [9, 10], CLUSTER, bs, previous_address=prev)
                manifest.close_on_grid(grid, images, [9, 10], previous_address=prev, previous_checksum=None)
                eng.synchronize()  # an unrelated wait does not take the refusal
                with pytest.raises(abi.TbcError) as err:  # the refusal is reported
                    grid.manifest_close_status()
                assert err.value.status == abi.TBC_ERR_BLOCK_INVALID
                grid.manifest_close_status()  # reported once
                got = grid.get_blocks([9, 10])
                assert not got[:, :16].any(), prev  # header checksums left zero
                res = eng.validate_blocks([grid.pointer(9), grid.pointer(10)], [0, 0], [9, 10])
                assert all(r == 1 for r in res), res  # invalid_checksum
            # an address reused after a checkpoint, verified from
            # its earlier block (6, closed above), refused again: its verified
            # byte is cleared, so a later close cannot link onto it.
            images = manifest.pack_blocks(_infos(20, 3), [6], CLUSTER, bs, previous_address=7)
            manifest.close_on_grid(grid, images, [6], previous_address=7, previous_checksum=None)
            with pytest.raises(abi.TbcError):
                grid.manifest_close_status()
            images = manifest.pack_blocks(_infos(20, 4), [11], CLUSTER, bs, previous_address=6)
            manifest.close_on_grid(grid, images, [11], previous_address=6, previous_checksum=None)
            with pytest.raises(abi.TbcError):  # 6 is no longer trusted: refused
                grid.manifest_close_status()
            assert not grid.get_blocks([6, 11])[:, :16].any()
        finally:
            grid.close()


class _DictStore:
    """The oracle's close_block into a host dict (the CPU side of the log tests)."""

    def __init__(self, bs):
        self.bs, self.grid, self.sums, self.closed = bs, {}, {}, []

    def close(self, infos, address, previous_address):
        imgs, sums = oracle.manifest_blocks(infos, [address], CLUSTER, self.bs,
                                            previous_checksum=self.sums.get(previous_address, 0),
                                            previous_address=previous_address)
        self.grid[address], self.sums[address] = imgs[0], sums[0]
        self.closed.append(address)

    def read(self, address):
        return self.grid[address]


def _drive_log(log, rng, half_bars: int, events_per_half_bar: int):
    """A random but valid event stream (insert, then update to invisible or a
    move, then remove), half-bar by half-bar, as Tree.compact_end appends:
    returns the model's live tables {address: encoded entry}."""
    from tigerbeetle_amd.tables import EVENT_INSERT, EVENT_REMOVE, EVENT_UPDATE, TableInfo
    live, invisible, next_addr = {}, {}, [10_000]
    op = 32
    for hb in range(half_bars):
        log.compact(op)
        for _ in range(events_per_half_bar):
            r = rng.random()
            if r < 0.45 or not live:
                a = next_addr[0]
                next_addr[0] += 1
                lo = int(rng.integers(0, 1 << 40))
                t = TableInfo(lo, lo + int(rng.integers(1, 1 << 20)), int(rng.integers(1, 1 << 62)) << 60 | a, a, op,
                              (1 << 64) - 1, int(rng.integers(1, 9000)), 8, int(rng.integers(0, 7)))
                e = t.encode(8, t.level, EVENT_INSERT, 16)
                live[a] = (t, e)
            elif r < 0.75:
                a = list(live)[int(rng.integers(0, len(live)))]
                t, _ = live[a]
                if rng.random() < 0.3 and t.level < 6:        # a move: update at the next level
                    t = TableInfo(t.key_min, t.key_max, t.checksum, a, t.snapshot_min, t.snapshot_max,
                                  t.value_count, 8, t.level + 1)
                    live[a] = (t, t.encode(8, t.level, EVENT_UPDATE, 16))
                    e = live[a][1]
                else:                                          # an input: snapshot_max set, then removed
                    t = TableInfo(t.key_min, t.key_max, t.checksum, a, t.snapshot_min, op + 15, t.value_count, 8,
                                  t.level)
                    e = t.encode(8, t.level, EVENT_UPDATE, 16)
                    del live[a]
                    invisible[a] = t
            elif invisible:
                a = list(invisible)[int(rng.integers(0, len(invisible)))]
                t = invisible.pop(a)
                e = t.encode(8, t.level, EVENT_REMOVE, 16)
            else:
                continue
            log.append(e)
        log.compact_end()
        op += 16
    return live, invisible


@pytest.mark.parametrize("seed", [1, 2])
def test_manifest_log_compaction_and_recovery(seed):
    """ManifestLog at test_min block size (30 entries a block) over many
    half-bars: blocks close when full, the oldest are compacted (latest
    extents re-appended, the rest dropped) and released; after a checkpoint,
    opening the log newest-first (ManifestLog.open) and replaying it
    chronologically (Forest.verify_tables_recovered's strategy 1) both give
    exactly the model's tables, and the extents cover them (verify_table_extents)."""
    from tigerbeetle_amd.forest import FreeSet
    rng = np.random.default_rng(seed)
    fs = FreeSet(1 << 16)
    store = _DictStore(4096)
    log = manifest.ManifestLog(store, fs, 4096)
    assert log.entry_count_max == 30
    live, invisible = _drive_log(log, rng, half_bars=300, events_per_half_bar=12)
    log.checkpoint()
    assert log.stats["blocks_compacted"] > 20 and log.stats["entries_dropped"] > 0
    blocks = [store.grid[a] for a in log.log_addresses]
    for b, blk in enumerate(blocks):  # the chain: each block links the one before it in the log
        prev_a = int(blk[160:168].view(np.uint64)[0])
        if b:
            assert prev_a == log.log_addresses[b - 1]
    opened = manifest.open_log(blocks)
    replayed = manifest.replay_log(blocks)
    want = {a: e for a, (t, e) in live.items()}
    want.update({a: t.encode(8, t.level, 2, 16) for a, t in invisible.items()})
    assert set(opened) == set(want) == set(log.table_extents)
    for a, e in want.items():
        assert np.array_equal(opened[a], e)
    assert sorted(int(e[96:104].view(np.uint64)[0]) for e in replayed.values()) == sorted(want)


def test_manifest_pace_production():
    # manifest_log.zig Pace for the production forest (21 trees, 1 MiB blocks)
    p = manifest.Pace(manifest.TREE_COUNT, manifest.TABLE_COUNT_MAX, 1, manifest.entry_count_max(1 << 20))
    assert (p.half_bar_append_blocks_max, p.half_bar_compact_blocks_max, p.log_blocks_full_max) == (1, 2, 293)
    assert p.log_blocks_cycle_max == 586 and p.log_blocks_max > p.log_blocks_cycle_max
    assert p.half_bar_compact_blocks(0, 100) == 0 and p.half_bar_compact_blocks(3, 100) == 2
    assert p.half_bar_compact_blocks(585, 100) == 2


def test_no_entries_no_blocks():
    # close_block asserts entry_count > 0 (manifest_log.zig:913): nothing to close
    assert manifest.pack_blocks(np.zeros((0, 128), np.uint8), [], CLUSTER, 4096) == []
    assert oracle.manifest_blocks(np.zeros((0, 128), np.uint8), [], CLUSTER, 4096) == ([], [])
