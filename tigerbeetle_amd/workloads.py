"""Synthetic table contents for tests and benchmarks (numpy, seeded).

Values are byte-exact TigerBeetle Values (src/tigerbeetle.zig:7-104,
src/lsm/groove.zig:48-76, src/lsm/composite_key.zig:17-46): keys are given
as little-endian u64 limbs (limb 0 least significant), the tombstone flag is
bit 63 of the value's timestamp.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .abi import KEY_COMPOSITE_U64, KEY_COMPOSITE_U128, KEY_ID_U128, KEY_TIMESTAMP, USAGE_SECONDARY_INDEX
from .trees import HEADER_SIZE, TreeSpec

TOMB = np.uint64(1 << 63)
MASK63 = np.uint64((1 << 63) - 1)


def nlimbs(tree: TreeSpec) -> int:
    return {KEY_TIMESTAMP: 1, KEY_ID_U128: 2, KEY_COMPOSITE_U64: 2, KEY_COMPOSITE_U128: 3}[tree.key_kind]


def random_keys(tree: TreeSpec, n: int, rng: np.random.Generator, field_max: int | None = None) -> list:
    """n random key limb arrays (not necessarily unique)."""
    L = nlimbs(tree)
    limbs = []
    for i in range(L):
        x = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n, dtype=np.uint64)
        limbs.append(x)
    if tree.key_kind != KEY_ID_U128:
        limbs[0] &= MASK63  # timestamps never carry the tombstone bit in the key
        limbs[0][limbs[0] == 0] = 1
    if field_max is not None and L > 1:
        limbs[1] = rng.integers(0, field_max, size=n, dtype=np.uint64)
        for i in range(2, L):
            limbs[i] = np.zeros(n, dtype=np.uint64)
    return limbs


def sort_keys(limbs: list) -> np.ndarray:
    """Permutation sorting keys ascending (stable)."""
    return np.lexsort(tuple(limbs), axis=0) if len(limbs) > 1 else np.argsort(limbs[0], kind="stable")


def unique_sorted_keys(tree: TreeSpec, n: int, rng: np.random.Generator, field_max=None) -> list:
    """n distinct keys, ascending."""
    out = None
    want = n
    while True:
        limbs = random_keys(tree, int(want * 1.05) + 16, rng, field_max)
        if out is not None:
            limbs = [np.concatenate([a, b]) for a, b in zip(out, limbs)]
        order = sort_keys(limbs)
        limbs = [l[order] for l in limbs]
        if len(limbs[0]) > 1:
            diff = np.zeros(len(limbs[0]), dtype=bool)
            diff[0] = True
            for l in limbs:
                diff[1:] |= l[1:] != l[:-1]
            limbs = [l[diff] for l in limbs]
        if len(limbs[0]) >= n:
            idx = np.sort(rng.choice(len(limbs[0]), size=n, replace=False))
            return [l[idx] for l in limbs]
        out = limbs
        want = n - len(limbs[0]) + 16


def values_from_keys(tree: TreeSpec, limbs: list, tomb: np.ndarray, rng: np.random.Generator) -> np.ndarray:
    """Build Values (n, value_size) uint8 for the given keys / tombstone flags."""
    n = len(limbs[0])
    vs = tree.value_size
    tomb = np.asarray(tomb, dtype=bool)
    out = np.zeros((n, vs), dtype=np.uint8)
    w = out.view(np.uint64)  # (n, vs/8)
    tbit = np.where(tomb, TOMB, np.uint64(0))
    if tree.key_kind == KEY_TIMESTAMP:
        # Object: random body; a tombstone is a zeroed Value with ts | bit63
        # (groove.zig:38-44).
        body = rng.integers(0, 1 << 63, size=(n, vs // 8), dtype=np.uint64)
        body[tomb] = 0
        w[:] = body
        w[:, tree.timestamp_offset // 8] = limbs[0] | tbit
    elif tree.key_kind == KEY_ID_U128:
        # IdTreeValue{id, timestamp, padding = 0} (groove.zig:48-76)
        w[:, 0] = limbs[0]
        w[:, 1] = limbs[1]
        ts = rng.integers(1, 1 << 62, size=n, dtype=np.uint64)
        w[:, 2] = ts | tbit
    elif tree.key_kind == KEY_COMPOSITE_U64:
        w[:, 0] = limbs[1]
        w[:, 1] = limbs[0] | tbit
    else:
        w[:, 0] = limbs[1]
        w[:, 1] = limbs[2]
        w[:, 2] = limbs[0] | tbit
    return out


def split_blocks(values: np.ndarray, vcm: int) -> list:
    return [values[i:i + vcm] for i in range(0, len(values), vcm)]


@dataclass
class JobInputs:
    tree: TreeSpec
    a_values: np.ndarray          # immutable: sorted (dups allowed); disk: strictly increasing
    a_immutable: bool
    b_tables: list                # list of (n_i, vs) arrays, each strictly increasing, disjoint, ascending
    drop_tombstones: bool

    def a_segments_host(self, vcm: int) -> list:
        return [self.a_values] if self.a_immutable else split_blocks(self.a_values, vcm)

    def b_blocks_host(self, vcm: int) -> list:
        blocks = []
        for t in self.b_tables:
            blocks.extend(split_blocks(t, vcm))
        return blocks


def make_job_inputs(tree: TreeSpec, rng: np.random.Generator, *, n_a: int, b_table_sizes: list,
                    a_immutable: bool, overlap: float = 0.2, dup_frac: float = 0.0,
                    tomb_frac: float = 0.0, drop_tombstones: bool = False,
                    field_max: int | None = None) -> JobInputs:
    """Random valid inputs for one compaction (respecting the reference's
    invariants, e.g. secondary-index put/remove pairing)."""
    secondary = tree.usage == USAGE_SECONDARY_INDEX
    n_b = int(sum(b_table_sizes))
    n_overlap = int(min(n_b, n_a) * overlap)
    n_a_unique = max(0, n_a - int(n_a * dup_frac)) if a_immutable else n_a
    n_a_unique = max(n_a_unique, n_overlap) if n_a else 0
    n_a_only = max(0, n_a_unique - n_overlap)
    universe = unique_sorted_keys(tree, n_b + n_a_only, rng, field_max)
    U = len(universe[0])
    perm = rng.permutation(U)
    b_idx = np.sort(perm[:n_b])
    a_only_idx = np.sort(perm[n_b:n_b + n_a_only])
    ov_idx = np.sort(rng.choice(b_idx, size=n_overlap, replace=False)) if n_overlap else np.zeros(0, dtype=np.int64)

    # B: never dropped; secondary-index B values are puts (tombstones cancel in A).
    b_tomb = np.zeros(n_b, dtype=bool) if secondary else rng.random(n_b) < tomb_frac
    b_limbs = [l[b_idx] for l in universe]
    b_values = values_from_keys(tree, b_limbs, b_tomb, rng)
    b_tables, o = [], 0
    for s in b_table_sizes:
        b_tables.append(b_values[o:o + s])
        o += s

    a_key_idx = np.sort(np.concatenate([a_only_idx, ov_idx]))
    if len(a_key_idx) == 0 or n_a == 0:
        return JobInputs(tree, np.zeros((0, tree.value_size), dtype=np.uint8), a_immutable, b_tables,
                         drop_tombstones)
    in_b = np.isin(a_key_idx, ov_idx)
    if secondary:
        # A survivor of a key present in B must be its removal (tombstone) and
        # vice versa; with drop_tombstones every surviving A tombstone must
        # cancel a B put (compaction.zig:729-731, 766-769).
        a_tomb = in_b.copy()
    else:
        a_tomb = rng.random(len(a_key_idx)) < tomb_frac
    reps = np.ones(len(a_key_idx), dtype=np.int64)
    if a_immutable and n_a > len(a_key_idx):
        extra = n_a - len(a_key_idx)
        if secondary:
            # add whole put/remove pairs in front of the survivor
            pairs = rng.choice(len(a_key_idx), size=max(1, extra // 2), replace=True)
            np.add.at(reps, pairs, 2)
        else:
            more = rng.choice(len(a_key_idx), size=extra, replace=True)
            np.add.at(reps, more, 1)
    keys_rep = np.repeat(a_key_idx, reps)
    # tombstone flags per run element: the run's last element carries a_tomb;
    # secondary runs alternate so adjacent pairs differ.
    run_pos = np.concatenate([np.arange(r)[::-1] for r in reps]) if len(reps) else np.zeros(0, dtype=np.int64)
    last_tomb = np.repeat(a_tomb, reps)
    if secondary:
        tomb_rep = np.where(run_pos % 2 == 0, last_tomb, ~last_tomb)
    else:
        tomb_rep = np.where(run_pos == 0, last_tomb, rng.random(len(keys_rep)) < tomb_frac)
    a_limbs = [l[keys_rep] for l in universe]
    a_values = values_from_keys(tree, a_limbs, tomb_rep, rng)
    return JobInputs(tree, a_values, a_immutable, b_tables, drop_tombstones)


def shuffle_for_memtable(values: np.ndarray, rng: np.random.Generator, tree: TreeSpec) -> np.ndarray:
    """An insertion order whose stable sort is `values` (duplicates keep their
    relative order, so 'last put wins' is preserved)."""
    n = len(values)
    if n == 0:
        return values
    # Interleave: random permutation of distinct-key groups keeps runs' order
    # only if we permute runs, not elements. Permute element order but restore
    # per-key order by a stable pass.
    order = rng.permutation(n)
    # stable fix-up: within each key run, the elements must appear in their
    # original relative order: sort positions of each run.
    keys = keys_of(values, tree)
    run_id = np.zeros(n, dtype=np.int64)
    if n > 1:
        newrun = np.zeros(n, dtype=bool)
        newrun[0] = True
        for l in keys:
            newrun[1:] |= l[1:] != l[:-1]
        run_id = np.cumsum(newrun) - 1
    pos = np.empty(n, dtype=np.int64)
    pos[order] = np.arange(n)  # pos[i] = new position of element i
    # for each run, assign its sorted set of positions to its elements in order
    idx_by_run = np.argsort(run_id, kind="stable")
    pos_sorted = pos[idx_by_run]
    # sort positions within runs
    runs = run_id[idx_by_run]
    key2 = np.lexsort((pos_sorted, runs))
    pos_fixed = np.empty(n, dtype=np.int64)
    pos_fixed[idx_by_run] = pos_sorted[key2]
    out = np.empty_like(values)
    out[pos_fixed] = values
    return out


def keys_of(values: np.ndarray, tree: TreeSpec) -> list:
    w = np.ascontiguousarray(values).view(np.uint64)
    if tree.key_kind == KEY_TIMESTAMP:
        return [w[:, tree.timestamp_offset // 8] & MASK63]
    if tree.key_kind == KEY_ID_U128:
        return [w[:, 0].copy(), w[:, 1].copy()]
    if tree.key_kind == KEY_COMPOSITE_U64:
        return [w[:, 1] & MASK63, w[:, 0].copy()]
    return [w[:, 2] & MASK63, w[:, 0].copy(), w[:, 1].copy()]


def addresses_for(count: int, rng: np.random.Generator, start: int = 1, fragment: float = 0.0) -> np.ndarray:
    """Ascending free addresses of a reservation (free_set.zig:302-345); with
    fragmentation some addresses in between are already acquired."""
    if fragment <= 0:
        return np.arange(start, start + count, dtype=np.uint64)
    out = []
    a = start
    while len(out) < count:
        if rng.random() >= fragment:
            out.append(a)
        a += 1
    return np.asarray(out, dtype=np.uint64)


def worst_case_blocks(tree: TreeSpec, n_values: int, block_size: int) -> int:
    lay = tree.layout(block_size)
    db = -(-n_values // lay["block_value_count_max"])
    tables = -(-db // lay["data_block_count_max"])
    return db + tables
