"""Host-side view of the tables a compaction produces (manifest metadata).

`ManifestNode.TableInfo` (src/lsm/schema.zig:489-509) is what the reference's
Manifest keeps per table and what `Compaction.Context` names an input table
by (TableInfoReference, src/lsm/compaction.zig:84-99): the index block's
address and checksum, the key range and the value count. The engine returns
one per output table (tbc_batch_result); a grid compaction takes them back as
`tbc_table_ref`s.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SNAPSHOT_LATEST = (1 << 64) - 1  # lsm.snapshot_latest (manifest.zig:43)


@dataclass(frozen=True)
class TableInfo:
    key_min: int
    key_max: int
    checksum: int
    address: int
    snapshot_min: int
    snapshot_max: int
    value_count: int
    tree_id: int
    level: int

    @classmethod
    def decode(cls, raw, key_size: int) -> "TableInfo":
        b = np.ascontiguousarray(raw, dtype=np.uint8).tobytes()
        assert len(b) == 128
        u64 = lambda o: int.from_bytes(b[o:o + 8], "little")  # noqa: E731
        return cls(key_min=int.from_bytes(b[0:key_size], "little"),
                   key_max=int.from_bytes(b[32:32 + key_size], "little"),
                   checksum=int.from_bytes(b[64:80], "little"),
                   address=u64(96), snapshot_min=u64(104), snapshot_max=u64(112),
                   value_count=int.from_bytes(b[120:124], "little"),
                   tree_id=int.from_bytes(b[124:126], "little"),
                   level=b[126] & 0x3f)

    def ref(self) -> tuple:
        """(index address, index checksum, value count): a tbc_table_ref."""
        return (self.address, self.checksum, self.value_count)

    def visible(self, snapshot: int = SNAPSHOT_LATEST) -> bool:
        """TableInfo.visible (manifest.zig:121-149)."""
        return self.snapshot_min <= snapshot <= self.snapshot_max


def key_of_value(value: np.ndarray, key_kind: int, timestamp_offset: int) -> int:
    """key_from_value as an integer (composite_key.zig:48-50, groove.zig:22-76)."""
    w = np.ascontiguousarray(value).view(np.uint64)
    mask = (1 << 63) - 1
    if key_kind == 0:
        return int(w[timestamp_offset // 8]) & mask
    if key_kind == 1:
        return int(w[0]) | int(w[1]) << 64
    if key_kind == 2:
        return (int(w[1]) & mask) | int(w[0]) << 64
    return (int(w[2]) & mask) | int(w[0]) << 64 | int(w[1]) << 128
