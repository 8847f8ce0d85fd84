"""Generate tests/golden/: committed input/output vectors for the compaction path.

    python tools/make_golden.py

The reference ships no golden block bytes (data/index block
bytes are "parity unpinned by reference tests"), so the goldens are produced
by the CPU oracle (oracle/tbc_oracle.c) after it has reproduced the
reference's own AEGIS-128L known-answer tests (src/vsr/checksum.zig:94-195,
checked in tests/test_oracle.py). Each case is test_min-shaped (4 KiB blocks,
config.zig:241-269) so the fixtures stay small while still spanning several
data blocks and tables. The files are data only (npz without pickles + JSON).

Layout:
  tests/golden/kats.json           the reference KATs (checksum.zig:94-195)
  tests/golden/cases.json          per-case metadata (tree, flags, sizes)
  tests/golden/case_<name>.npz     a, b (concatenated B tables), b_sizes,
                                   addresses, images (disk images of the output
                                   blocks concatenated), image_sizes, infos
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402  (test infrastructure: the checker that makes the vectors)
from tigerbeetle_amd import trees, workloads  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
BS = 4096
CLUSTER = 0x0123456789ABCDEF_FEDCBA9876543210
SNAPSHOT_MIN = 48  # snapshot_min_for_table_output(op_min=32)

# (name, tree, level_b, make_job_inputs kwargs)
CASES = [
    ("id_disk_a", "transfers.id", 1,
     dict(n_a=900, b_table_sizes=[400, 500, 200], a_immutable=False, overlap=0.3)),
    ("id_immutable_drop", "accounts.id", 6,
     dict(n_a=1100, b_table_sizes=[600], a_immutable=True, dup_frac=0.2, tomb_frac=0.1, drop_tombstones=True,
          overlap=0.5)),
    ("object_128_tombstones", "transfers.timestamp", 2,
     dict(n_a=300, b_table_sizes=[60, 90, 40], a_immutable=True, dup_frac=0.3, tomb_frac=0.2, overlap=0.4)),
    ("object_16_b_only", "posted.timestamp", 3,
     dict(n_a=0, b_table_sizes=[700, 500], a_immutable=False, tomb_frac=0.1)),
    ("object_256_last_level", "account_history.timestamp", 6,
     dict(n_a=150, b_table_sizes=[50, 70], a_immutable=True, dup_frac=0.2, tomb_frac=0.2, drop_tombstones=True,
          overlap=0.3)),
    ("secondary_u256_cancel", "transfers.debit_account_id", 1,
     dict(n_a=1300, b_table_sizes=[400, 300], a_immutable=True, dup_frac=0.4, drop_tombstones=True,
          overlap=0.3)),
    ("secondary_u128", "accounts.ledger", 2,
     dict(n_a=1200, b_table_sizes=[900], a_immutable=True, dup_frac=0.3, overlap=0.5)),
    ("single_value", "transfers.amount", 1,
     dict(n_a=1, b_table_sizes=[], a_immutable=True)),
]


def disk_image(block: np.ndarray) -> np.ndarray:
    size = int(block[96:100].view(np.uint32)[0])
    return block[: -(-size // trees.SECTOR_SIZE) * trees.SECTOR_SIZE]


def case_tree(tree_name: str) -> trees.TreeSpec:
    base = trees.BY_NAME[tree_name]
    # multi-block, multi-table outputs on 4 KiB blocks
    return trees.with_table_size(base, 3 * (BS - 256) // base.value_size + 5)


def main() -> None:
    oracle.build()
    os.makedirs(OUT, exist_ok=True)
    kats = {
        "source": "src/vsr/checksum.zig:94-112 (test vectors), :146-195 (stability)",
        "zero16_le_hex": "f72ad48dd05dd1656133101cd4be3a26",  # checksum.zig:100-104: @byteSwap of the u128 literal
        "empty_u128": "0x49F174618255402DE6E7E3C40D60CC83",
        "stability_hash_u128": "0x82dcaacf4875b279446825b6830d1263",
    }
    json.dump(kats, open(os.path.join(OUT, "kats.json"), "w"), indent=1)
    meta = []
    for i, (name, tree_name, level_b, kw) in enumerate(CASES):
        spec = case_tree(tree_name)
        rng = np.random.default_rng(0x601D + i)
        ji = workloads.make_job_inputs(spec, rng, **kw)
        n = len(ji.a_values) + sum(len(t) for t in ji.b_tables)
        addrs = workloads.addresses_for(workloads.worst_case_blocks(spec, n, BS) + 2, rng, 100 + 10 * i, 0.15)
        t = oracle.tree(spec.tree_id, spec.key_kind, spec.usage, spec.value_size, spec.timestamp_offset,
                        spec.value_count_max, BS)
        vcm = t.block_value_count_max
        r = oracle.compact(t, ji.a_segments_host(vcm), ji.b_blocks_host(vcm), a_immutable=ji.a_immutable,
                           drop_tombstones=ji.drop_tombstones, level_b=level_b, cluster=CLUSTER,
                           snapshot_min=SNAPSHOT_MIN, addresses=addrs)
        assert r.status == 0
        images = [disk_image(b) for b in r.blocks]
        b_all = np.concatenate(ji.b_tables) if ji.b_tables else np.zeros((0, spec.value_size), np.uint8)
        np.savez_compressed(
            os.path.join(OUT, f"case_{name}.npz"),
            a=ji.a_values, b=b_all, b_sizes=np.array([len(x) for x in ji.b_tables], dtype=np.int64),
            addresses=np.asarray(addrs, dtype=np.uint64),
            images=np.concatenate(images) if images else np.zeros(0, np.uint8),
            image_sizes=np.array([len(x) for x in images], dtype=np.int64),
            infos=r.table_infos)
        meta.append(dict(name=name, tree=tree_name, value_count_max=spec.value_count_max, level_b=level_b,
                         a_immutable=bool(ji.a_immutable), drop_tombstones=bool(ji.drop_tombstones),
                         block_size=BS, cluster=hex(CLUSTER), snapshot_min=SNAPSHOT_MIN,
                         value_count=int(r.value_count), data_block_count=int(r.data_block_count),
                         table_count=len(r.table_infos), block_count=len(r.blocks)))
        print(f"{name}: {n} values in -> {r.value_count} out, {len(r.blocks)} blocks, {len(r.table_infos)} tables")
    json.dump({"generator": "tools/make_golden.py", "oracle": "oracle/tbc_oracle.c", "cases": meta},
              open(os.path.join(OUT, "cases.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
