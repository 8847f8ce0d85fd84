"""TigerBeetle's forest: the 21 LSM trees and their table parameters.

Restates the grooves of src/state_machine.zig:167-273 (value_count_max per
tree), tree ids (src/state_machine.zig:78-111), Value layouts
(src/tigerbeetle.zig:7-104, src/lsm/groove.zig:22-134,
src/lsm/composite_key.zig:7-70) and the production config
(src/config.zig:130-185: block_size 1 MiB, lsm_batch_multiple 32).
"""
from __future__ import annotations

from dataclasses import dataclass

from .abi import (KEY_COMPOSITE_U64, KEY_COMPOSITE_U128, KEY_ID_U128, KEY_TIMESTAMP,
                  USAGE_GENERAL, USAGE_SECONDARY_INDEX, Tree)

BLOCK_SIZE = 1 << 20            # config.zig:139
HEADER_SIZE = 256               # message_header.zig:68
SECTOR_SIZE = 4096              # constants.zig:418
LSM_BATCH_MULTIPLE = 32         # config.zig:142
LSM_GROWTH_FACTOR = 8           # config.zig:141
LSM_LEVELS = 7                  # config.zig:140
MESSAGE_SIZE_MAX = 1 << 20      # config.zig:137
# StateMachine.constants.batch_max (state_machine.zig:53-76): body / max(event, result)
BATCH_MAX_CREATE_TRANSFERS = (MESSAGE_SIZE_MAX - HEADER_SIZE) // 128  # 8190
BATCH_MAX_CREATE_ACCOUNTS = (MESSAGE_SIZE_MAX - HEADER_SIZE) // 128   # 8190


@dataclass(frozen=True)
class TreeSpec:
    name: str
    tree_id: int
    key_kind: int
    usage: int
    value_size: int
    timestamp_offset: int
    value_count_max: int

    def ctype(self) -> Tree:
        return Tree(self.tree_id, self.key_kind, self.usage, self.value_size, self.timestamp_offset,
                    self.value_count_max)

    @property
    def key_size(self) -> int:
        return {KEY_TIMESTAMP: 8, KEY_ID_U128: 16, KEY_COMPOSITE_U64: 16, KEY_COMPOSITE_U128: 32}[self.key_kind]

    def layout(self, block_size: int = BLOCK_SIZE) -> dict:
        """TableType.layout (table.zig:107-129) + TableIndex.init (schema.zig:119-157)."""
        vcm = (block_size - HEADER_SIZE) // self.value_size
        dbcm = -(-self.value_count_max // vcm)
        ks = self.key_size
        return {
            "block_value_count_max": vcm,
            "data_block_count_max": dbcm,
            "block_count_max": dbcm + 1,
            "index_size": HEADER_SIZE + dbcm * (32 + 2 * ks + 8),
        }


def _id(name, tid, vcm):
    return TreeSpec(name, tid, KEY_ID_U128, USAGE_GENERAL, 32, 16, vcm)


def _c128(name, tid, vcm):
    return TreeSpec(name, tid, KEY_COMPOSITE_U128, USAGE_SECONDARY_INDEX, 32, 16, vcm)


def _c64(name, tid, vcm):
    return TreeSpec(name, tid, KEY_COMPOSITE_U64, USAGE_SECONDARY_INDEX, 16, 8, vcm)


def _obj(name, tid, vs, ts, vcm):
    return TreeSpec(name, tid, KEY_TIMESTAMP, USAGE_GENERAL, vs, ts, vcm)


_T = LSM_BATCH_MULTIPLE * BATCH_MAX_CREATE_TRANSFERS  # 262,080
_A = LSM_BATCH_MULTIPLE * BATCH_MAX_CREATE_ACCOUNTS   # 262,080
_A_TS = LSM_BATCH_MULTIPLE * max(BATCH_MAX_CREATE_ACCOUNTS, 2 * BATCH_MAX_CREATE_TRANSFERS)  # 524,160

# Account (tigerbeetle.zig:7-40): timestamp at byte 120. Transfer (80-104): 120.
# PostedGrooveValue (state_machine.zig:251-262): timestamp at 0, 16 bytes.
# AccountHistoryGrooveValue (state_machine.zig:280-301): timestamp at 160, 256 bytes.
TREES = [
    _id("accounts.id", 1, _A),
    _c128("accounts.user_data_128", 2, _A),
    _c64("accounts.user_data_64", 3, _A),
    _c64("accounts.user_data_32", 4, _A),
    _c64("accounts.ledger", 5, _A),
    _c64("accounts.code", 6, _A),
    _obj("accounts.timestamp", 7, 128, 120, _A_TS),
    _id("transfers.id", 8, _T),
    _c128("transfers.debit_account_id", 9, _T),
    _c128("transfers.credit_account_id", 10, _T),
    _c128("transfers.amount", 11, _T),
    _c128("transfers.pending_id", 12, _T),
    _c128("transfers.user_data_128", 13, _T),
    _c64("transfers.user_data_64", 14, _T),
    _c64("transfers.user_data_32", 15, _T),
    _c64("transfers.timeout", 16, _T),
    _c64("transfers.ledger", 17, _T),
    _c64("transfers.code", 18, _T),
    _obj("transfers.timestamp", 19, 128, 120, _T),
    _obj("posted.timestamp", 20, 16, 0, _T),
    _obj("account_history.timestamp", 21, 256, 160, _T),
]
BY_NAME = {t.name: t for t in TREES}
BY_ID = {t.tree_id: t for t in TREES}


def snapshot_min_for_table_output(op_min: int) -> int:
    """compaction.zig:981-985."""
    assert op_min > 0 and op_min % (LSM_BATCH_MULTIPLE // 2) == 0
    return op_min + LSM_BATCH_MULTIPLE // 2


def with_table_size(spec: TreeSpec, value_count_max: int) -> TreeSpec:
    """The same tree with another Table.value_count_max (e.g. test configs)."""
    from dataclasses import replace
    return replace(spec, value_count_max=value_count_max)


# config.zig:241-269 test_min: block_size = sector_size, lsm_batch_multiple = 4,
# message_size_max = message_size_max_min(4) = 4096 -> batch_max = 30.
TEST_MIN_BLOCK_SIZE = 4096
TEST_MIN_BATCH = (4096 - HEADER_SIZE) // 128
TEST_MIN_TREES = [with_table_size(t, 4 * TEST_MIN_BATCH * (2 if t.tree_id == 7 else 1)) for t in TREES]
