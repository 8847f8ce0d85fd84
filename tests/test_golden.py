"""Committed golden vectors (tests/golden/, made by tools/make_golden.py).

CPU: the oracle reproduces every fixture byte for byte, every fixture block's
checksums verify, and the fixture values equal the independent Python
restatement of compaction.zig (helpers.model_merge). GPU: libtbc.so
reproduces every fixture, all cases in one batch, through the C ABI.
"""
import json
import os

import numpy as np
import pytest

from helpers import HEADER, model_merge
from tigerbeetle_amd import trees, workloads

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(GOLDEN, "cases.json")))["cases"]


def load(meta):
    d = np.load(os.path.join(GOLDEN, f"case_{meta['name']}.npz"))  # allow_pickle=False (default)
    spec = trees.with_table_size(trees.BY_NAME[meta["tree"]], meta["value_count_max"])
    b_tables, o = [], 0
    for s in d["b_sizes"]:
        b_tables.append(d["b"][o:o + int(s)])
        o += int(s)
    ji = workloads.JobInputs(spec, d["a"], meta["a_immutable"], b_tables, meta["drop_tombstones"])
    images, o = [], 0
    for s in d["image_sizes"]:
        images.append(d["images"][o:o + int(s)])
        o += int(s)
    return ji, d["addresses"], images, d["infos"]


def disk_image(block):
    size = int(block[96:100].view(np.uint32)[0])
    return block[: -(-size // trees.SECTOR_SIZE) * trees.SECTOR_SIZE]


def test_kats_fixture_matches_oracle(oracle_lib):
    k = json.load(open(os.path.join(GOLDEN, "kats.json")))
    assert oracle_lib.checksum(bytes(16)) == int.from_bytes(bytes.fromhex(k["zero16_le_hex"]), "little")
    assert oracle_lib.checksum(b"") == int(k["empty_u128"], 16)


@pytest.mark.parametrize("meta", META, ids=[m["name"] for m in META])
def test_oracle_reproduces_golden(oracle_lib, meta):
    ji, addrs, images, infos = load(meta)
    bs = meta["block_size"]
    t = oracle_lib.tree(ji.tree.tree_id, ji.tree.key_kind, ji.tree.usage, ji.tree.value_size,
                        ji.tree.timestamp_offset, ji.tree.value_count_max, bs)
    vcm = t.block_value_count_max
    r = oracle_lib.compact(t, ji.a_segments_host(vcm), ji.b_blocks_host(vcm), a_immutable=ji.a_immutable,
                           drop_tombstones=ji.drop_tombstones, level_b=meta["level_b"],
                           cluster=int(meta["cluster"], 16), snapshot_min=meta["snapshot_min"], addresses=addrs)
    assert r.status == 0 and len(r.blocks) == len(images) == meta["block_count"]
    for got, want in zip(r.blocks, images):
        assert np.array_equal(disk_image(got), want)
    assert np.array_equal(r.table_infos, infos)
    # independent checks on the fixture itself
    vals = [img[HEADER:int(img[96:100].view(np.uint32)[0])].reshape(-1, ji.tree.value_size)
            for img in images if img[240] == 5]
    got_vals = np.concatenate(vals) if vals else np.zeros((0, ji.tree.value_size), np.uint8)
    assert np.array_equal(got_vals, model_merge(ji))
    for img in images:
        size = int(img[96:100].view(np.uint32)[0])
        assert oracle_lib.checksum(img[256:size].tobytes()) == int.from_bytes(img[32:48].tobytes(), "little")
        assert oracle_lib.checksum(img[16:256].tobytes()) == int.from_bytes(img[0:16].tobytes(), "little")
        assert not img[size:].any()  # zeroed sector tail (grid.zig:686)


@pytest.mark.gpu
def test_gpu_reproduces_golden(engine_small):
    from helpers import gpu_run
    loaded = [load(m) for m in META]
    by_level = {}
    for m, x in zip(META, loaded):
        by_level.setdefault((m["level_b"], m["cluster"], m["snapshot_min"]), []).append((m, x))
    for (level_b, cluster, snap), group in by_level.items():
        results, _ = gpu_run(engine_small, [x[0] for _, x in group], 4096, [x[1] for _, x in group],
                             level_b=level_b, cluster=int(cluster, 16), snapshot_min=snap)
        for (m, (ji, addrs, images, infos)), (r, ginfos, blocks) in zip(group, results):
            assert r.status == 0, m["name"]
            assert (r.value_count, r.block_count, r.table_count) == \
                (m["value_count"], m["block_count"], m["table_count"]), m["name"]
            for i, (g, w) in enumerate(zip(blocks, images)):
                assert np.array_equal(disk_image(g), w), f"{m['name']}: block {i}"
            assert np.array_equal(ginfos, infos), m["name"]
