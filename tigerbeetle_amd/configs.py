"""BASELINE.json workloads as seeded synthetic compaction jobs.

Every generator is deterministic in (config, job id), so any rank can build
any job without communication, and jobs are produced lazily (one job's host
arrays at a time) to keep host memory bounded at the 1B-value scale.

  config 2  transfers.id L0->L1: 1 disk A table + 8 full B tables of unique
            uniform-random u128 ids (IdTreeValue, 32 B), no dups/tombstones.
  config 3  secondary indexes transfers.debit_account_id / credit_account_id
            (CompositeKey(u128), 32 B): the bar's mutable table (262,080
            values, account id Zipf(1.1) over 10,000 accounts, timestamps
            monotone) arrives UNSORTED and is sorted on the device
            (TableMemory.sort) before its immutable->L0 compaction against 8
            L0 tables; 1% of the bar's puts are removed again (half inside the
            bar -> put/remove pairs cancel in fill_immutable_values, half
            removing an older put that lives in B -> both dropped by the
            secondary-index merge rule). Two jobs in every 7 are the
            sequential leg: the same index trees with an
            increasing field and monotone timestamps (job % 7 == 5: the
            memtable arrives sorted and its keys lie above every older table,
            so it flushes with no B and the deeper levels move), and the
            transfers.timestamp object tree (Transfer, 128 B; job % 7 == 6),
            likewise a pure flush.
  config 4  full groove compaction (one forest unit per GPU, 21 jobs): the
            bar-end immutable->L0 compaction of the 11 trees a create_transfers
            bar feeds (10 transfer trees — pending_id/timeout are 0 and not
            indexed, groove.zig:928-934 — plus the accounts object tree, 2
            updates per transfer over 10,000 accounts), each memtable sorted
            on the device when it arrives unsorted, and one L1->L2 disk
            compaction (1 A + 4 B tables) per transfer tree. Jobs differ in
            tree, key kind and size; ranks get whole jobs by bytes (LPT).
  config 5  accounts.timestamp object tree (Account, 128 B), last level:
            disk A = 1 table (524,160 newer versions of uniformly chosen
            existing keys, 1% tombstones) into 8 last-level B tables;
            drop_tombstones = true, level_b = 6.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import trees, workloads
from .workloads import TOMB

CONFIG2_SEED = 0x7B0002
CONFIG3_SEED = 0x7B0003
CONFIG5_SEED = 0x7B0005
TABLE_T = trees.BY_NAME["transfers.id"].value_count_max               # 262,080
TABLE_A_TS = trees.BY_NAME["accounts.timestamp"].value_count_max      # 524,160
ACCOUNTS = 10_000


@dataclass
class JobSpec:
    tree: trees.TreeSpec
    a: np.ndarray             # (n, vs) uint8; immutable: insertion order if a_unsorted
    a_immutable: bool
    a_unsorted: bool          # the memtable must be sorted (TableMemory.sort) first
    b_tables: list            # [(n_i, vs) uint8], ascending, disjoint
    drop_tombstones: bool
    level_b: int
    # TBC_COMPACTION_UNIQUE_KEYS: the tree's keys are never repeated or removed
    # (ids, immutable Transfers' object and index trees), so every value
    # survives and the engine may start every block's chain before merging.
    unique_keys: bool = False

    @property
    def input_values(self) -> int:
        return len(self.a) + sum(len(t) for t in self.b_tables)

    @property
    def input_bytes(self) -> int:
        return self.input_values * self.tree.value_size


def config2_job(job: int, n_b_tables: int = 8) -> JobSpec:
    """One transfers.id L0->L1 compaction (BASELINE configs[1])."""
    rng = np.random.default_rng(CONFIG2_SEED + job)
    n = TABLE_T * (n_b_tables + 1)
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
    a_idx = np.sort(rng.choice(n, size=TABLE_T, replace=False))
    mask = np.zeros(n, dtype=bool)
    mask[a_idx] = True
    a = vals[mask]
    b = vals[~mask]
    return JobSpec(trees.BY_NAME["transfers.id"], a, False, False,
                   [b[i * TABLE_T:(i + 1) * TABLE_T] for i in range(n_b_tables)], False, 1, unique_keys=True)


def _zipf_accounts(rng, n: int, s: float = 1.1) -> np.ndarray:
    ranks = np.arange(1, ACCOUNTS + 1, dtype=np.float64)
    p = ranks ** -s
    p /= p.sum()
    ids = rng.choice(ACCOUNTS, size=n, p=p).astype(np.uint64) + np.uint64(1)
    return ids


def _composite128(field: np.ndarray, ts: np.ndarray, tomb: np.ndarray) -> np.ndarray:
    """CompositeKey(u128){field, timestamp (| tombstone bit), padding 0}
    (composite_key.zig:17-46); field < 2^64 here (account ids)."""
    v = np.zeros((len(field), 32), dtype=np.uint8)
    w = v.view(np.uint64)
    w[:, 0] = field
    w[:, 2] = ts | np.where(tomb, TOMB, np.uint64(0))
    return v


def _sorted_composite(v: np.ndarray) -> np.ndarray:
    w = v.view(np.uint64)
    return v[np.lexsort((w[:, 2] & workloads.MASK63, w[:, 0], w[:, 1]))]  # field hi, field lo, ts (stable)


def config3_job(job: int, n_b_tables: int = 8) -> JobSpec:
    """One bar-end job of config 3 (BASELINE configs[2])."""
    rng = np.random.default_rng(CONFIG3_SEED + job)
    bar_ts0 = np.uint64(1 + (job + n_b_tables) * 4 * TABLE_T)  # later jobs are later bars
    if job % 7 == 6:
        # Sequential: transfers.timestamp, already-sorted memtable, empty L0.
        spec = trees.BY_NAME["transfers.timestamp"]
        ts = bar_ts0 + np.arange(TABLE_T, dtype=np.uint64)
        a = workloads.values_from_keys(spec, [ts], np.zeros(TABLE_T, dtype=bool), rng)
        return JobSpec(spec, a, True, False, [], False, 0, unique_keys=True)
    spec = trees.BY_NAME["transfers.debit_account_id" if job % 2 == 0 else "transfers.credit_account_id"]
    if job % 7 == 5:
        # Sequential secondary index: each new account's transfers in order
        # (four per account), fields above every older table's: the
        # memtable is already in key order and overlaps no L0 table.
        ts = bar_ts0 + np.arange(TABLE_T, dtype=np.uint64)
        field = np.uint64(1 + (job + n_b_tables) * TABLE_T) + np.arange(TABLE_T, dtype=np.uint64) // np.uint64(4)
        a = _composite128(field, ts, np.zeros(TABLE_T, dtype=bool))
        return JobSpec(spec, a, True, False, [], False, 0, unique_keys=True)
    # B: 8 L0 tables of older puts (timestamps before this bar), sorted, cut.
    nb = n_b_tables * TABLE_T
    b_ts = np.uint64(1) + rng.choice(int(bar_ts0) - 1, size=nb, replace=False).astype(np.uint64)
    b_all = _sorted_composite(_composite128(_zipf_accounts(rng, nb), b_ts, np.zeros(nb, dtype=bool)))
    b_tables = [b_all[i * TABLE_T:(i + 1) * TABLE_T] for i in range(n_b_tables)]
    # The bar: 262,080 index updates in timestamp order (insertion order).
    n_rm = TABLE_T // 100
    n_put = TABLE_T - n_rm
    put_ts = bar_ts0 + np.arange(n_put, dtype=np.uint64)
    put_field = _zipf_accounts(rng, n_put)
    ins = [_composite128(put_field, put_ts, np.zeros(n_put, dtype=bool))]
    # removes of puts inside this bar (appended after their put: insertion order)
    k_in = n_rm // 2
    victims = rng.choice(n_put, size=k_in, replace=False)
    ins.append(_composite128(put_field[victims], put_ts[victims], np.ones(k_in, dtype=bool)))
    # removes of older puts that live in B
    k_b = n_rm - k_in
    bw = b_all.view(np.uint64)
    old = rng.choice(nb, size=k_b, replace=False)
    ins.append(_composite128(bw[old, 0].copy(), bw[old, 2].copy(), np.ones(k_b, dtype=bool)))
    a = np.concatenate(ins)
    # Interleave removes after their puts: a random insertion order that keeps
    # each (field, ts) run in put-then-remove order (last put wins).
    a = workloads.shuffle_for_memtable(_sorted_composite(a), rng, spec)
    return JobSpec(spec, a, True, True, b_tables, False, 0)


def config5_job(job: int, n_b_tables: int = 8) -> JobSpec:
    """One last-level accounts.timestamp compaction (BASELINE configs[4])."""
    rng = np.random.default_rng(CONFIG5_SEED + job)
    spec = trees.BY_NAME["accounts.timestamp"]
    nb = n_b_tables * TABLE_A_TS
    # disjoint key range per job; strictly increasing timestamps with gaps
    base = np.uint64(1 + job * nb * 4)
    keys = base + np.cumsum(rng.integers(1, 4, size=nb, dtype=np.uint64))
    b_all = np.empty((nb, 128), dtype=np.uint8)
    bw = b_all.view(np.uint64)
    bw[:] = rng.integers(0, 1 << 63, size=(nb, 16), dtype=np.uint64)
    bw[:, 15] = keys  # timestamp at byte 120 (tigerbeetle.zig:7-40)
    a_idx = np.sort(rng.choice(nb, size=TABLE_A_TS, replace=False))
    tomb = rng.random(TABLE_A_TS) < 0.01
    a = np.empty((TABLE_A_TS, 128), dtype=np.uint8)
    aw = a.view(np.uint64)
    aw[:] = rng.integers(0, 1 << 63, size=(TABLE_A_TS, 16), dtype=np.uint64)
    aw[tomb] = 0  # tombstone = zeroed Value with ts | bit63 (groove.zig:38-44)
    aw[:, 15] = keys[a_idx] | np.where(tomb, TOMB, np.uint64(0))
    return JobSpec(spec, a, False, False, [b_all[i * TABLE_A_TS:(i + 1) * TABLE_A_TS] for i in range(n_b_tables)],
                   True, 6)


CONFIG4_SEED = 0x7B0004
# The 11 trees a create_transfers bar feeds.
FOREST_BAR = ["transfers.id", "transfers.timestamp", "transfers.debit_account_id", "transfers.credit_account_id",
              "transfers.amount", "transfers.user_data_128", "transfers.user_data_64", "transfers.user_data_32",
              "transfers.ledger", "transfers.code", "accounts.timestamp"]
FOREST_DEEP = FOREST_BAR[:10]
FOREST_JOBS = len(FOREST_BAR) + len(FOREST_DEEP)  # 21 per forest unit
L0_TABLES = 2


def _bar_fields(name: str, rng, n: int) -> np.ndarray:
    """Indexed field of n transfers (benchmark_load.zig:291-313 shapes)."""
    if name in ("transfers.debit_account_id", "transfers.credit_account_id"):
        return rng.integers(1, ACCOUNTS + 1, size=n, dtype=np.uint64)
    if name == "transfers.amount":
        return np.maximum(1, rng.exponential(10_000, size=n)).astype(np.uint64)
    if name == "transfers.ledger":
        return np.ones(n, dtype=np.uint64)
    if name == "transfers.code":
        return rng.integers(1, 100, size=n, dtype=np.uint64)
    if name == "transfers.user_data_32":
        return rng.integers(0, 1 << 32, size=n, dtype=np.uint64)
    return rng.integers(0, 1 << 63, size=n, dtype=np.uint64)


def _bar_values(spec: trees.TreeSpec, name: str, rng, ts: np.ndarray, ids: np.ndarray) -> np.ndarray:
    n = len(ts)
    if name == "transfers.id":
        v = np.zeros((n, 32), dtype=np.uint8)
        w = v.view(np.uint64)
        w[:, 0] = ids
        w[:, 2] = ts
        return v
    if name == "transfers.timestamp":
        return workloads.values_from_keys(spec, [ts], np.zeros(n, dtype=bool), rng)
    field = _bar_fields(name, rng, n)
    if spec.key_kind == workloads.KEY_COMPOSITE_U64:
        return workloads.values_from_keys(spec, [ts, field], np.zeros(n, dtype=bool), rng)
    return workloads.values_from_keys(spec, [ts, field, np.zeros(n, dtype=np.uint64)], np.zeros(n, dtype=bool), rng)


def _sorted_by_key(spec: trees.TreeSpec, v: np.ndarray) -> np.ndarray:
    return v[workloads.sort_keys(workloads.keys_of(v, spec))]


def config4_job(job: int) -> JobSpec:
    """Job `job` of the forest units (BASELINE configs[3]): unit = job // 21."""
    unit, k = divmod(job, FOREST_JOBS)
    rng = np.random.default_rng(CONFIG4_SEED + job)
    n = TABLE_T
    if k < len(FOREST_BAR):
        name = FOREST_BAR[k]
        spec = trees.BY_NAME[name]
        bar = unit + L0_TABLES + 1  # bars before this one fill L0
        if name == "accounts.timestamp":
            # 2 updates per transfer over 10,000 accounts (timestamps 1..10k),
            # insertion order = update order; L0 holds the previous versions.
            acc_ts = rng.integers(1, ACCOUNTS + 1, size=2 * n, dtype=np.uint64)
            a = workloads.values_from_keys(spec, [acc_ts], np.zeros(2 * n, dtype=bool), rng)
            b = workloads.values_from_keys(spec, [np.arange(1, ACCOUNTS + 1, dtype=np.uint64)],
                                           np.zeros(ACCOUNTS, dtype=bool), rng)
            return JobSpec(spec, a, True, True, [b], False, 0)
        ts0 = np.uint64(ACCOUNTS + 1 + bar * n)
        ts = ts0 + np.arange(n, dtype=np.uint64)
        ids = np.uint64(1 + bar * n) + np.arange(n, dtype=np.uint64)
        a = _bar_values(spec, name, rng, ts, ids)
        unsorted = bool(len(a) > 1 and workloads.sort_keys(workloads.keys_of(a, spec))[:-1].tolist()
                        != list(range(len(a) - 1)))
        # L0: the L0_TABLES previous bars of the same tree, merged and cut.
        old_ts = np.uint64(ACCOUNTS + 1 + (bar - L0_TABLES) * n) + np.arange(L0_TABLES * n, dtype=np.uint64)
        old_ids = np.uint64(1 + (bar - L0_TABLES) * n) + np.arange(L0_TABLES * n, dtype=np.uint64)
        b_all = _sorted_by_key(spec, _bar_values(spec, name, rng, old_ts, old_ids))
        # Transfers are immutable: their trees' bar-end keys are all new.
        return JobSpec(spec, a, True, unsorted, [b_all[i * n:(i + 1) * n] for i in range(L0_TABLES)], False, 0,
                       unique_keys=True)
    name = FOREST_DEEP[k - len(FOREST_BAR)]
    spec = trees.BY_NAME[name]
    ji = workloads.make_job_inputs(spec, rng, n_a=n, b_table_sizes=[n] * 4, a_immutable=False, overlap=0.05,
                                   tomb_frac=0.01 if spec.usage == 0 else 0.0)
    return JobSpec(spec, ji.a_values, False, False, ji.b_tables, False, 2)


def job_bytes(config: int, job: int) -> int:
    """Input bytes of a job without generating it (for the byte-balanced shard plan)."""
    if config == 2:
        return 9 * TABLE_T * 32
    if config == 3:
        return TABLE_T * (128 if job % 7 == 6 else 32 if job % 7 == 5 else 9 * 32)
    if config == 5:
        return 9 * TABLE_A_TS * 128
    k = job % FOREST_JOBS
    if k < len(FOREST_BAR):
        name = FOREST_BAR[k]
        if name == "accounts.timestamp":
            return (2 * TABLE_T + ACCOUNTS) * 128
        return (1 + L0_TABLES) * TABLE_T * trees.BY_NAME[name].value_size
    return 5 * TABLE_T * trees.BY_NAME[FOREST_DEEP[k - len(FOREST_BAR)]].value_size


def presorted(config: int, job: int) -> bool:
    """Whether the job's A needs no device sort first (a key-range split
    stages sorted ranges)."""
    if config == 3:
        return job % 7 in (5, 6)
    if config == 4:
        k = job % FOREST_JOBS
        return k >= len(FOREST_BAR) or FOREST_BAR[k] in ("transfers.id", "transfers.timestamp")
    return True


GENERATORS = {2: config2_job, 3: config3_job, 4: config4_job, 5: config5_job}
# --strong: the whole problem BASELINE states, divided over the GPUs (config 5:
# 216 x 4.7M = 1.02B Account values).
STRONG_JOBS = {2: 28, 3: 28, 4: FOREST_JOBS, 5: 216}
DEFAULT_JOBS = {2: 28, 3: 28, 4: FOREST_JOBS, 5: 27}
DESCRIPTION = {
    2: "transfers.id L0->L1 compaction, 28 jobs x (1 A + 8 B tables) per GPU, 64M u128 keys, 1 MiB blocks",
    3: "bar end of transfers.debit/credit_account_id (Zipf 1.1 over 10k accounts, unsorted memtable sorted on "
       "device, 1% put/remove pairs) + sequential legs (index trees with increasing fields, transfers.timestamp: "
       "already sorted flushes), 28 jobs per GPU",
    4: "full groove compaction: bar-end immutable->L0 of the 11 trees a create_transfers bar feeds (+ on-device "
       "memtable sorts) and one L1->L2 job per transfer tree, 21 jobs of 4 key kinds per GPU, sharded by bytes",
    5: "accounts.timestamp last-level compaction (Account 128 B, 1% tombstones dropped), 27 jobs x 4.7M values "
       "per GPU (1B values over 8 GPUs)",
}
