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
# schema.ManifestNode.Event (schema.zig:511-516)
EVENT_INSERT, EVENT_UPDATE, EVENT_REMOVE = 1, 2, 3


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

    @staticmethod
    def event_of(raw) -> int:
        """The label's event (schema.zig:518-530) of an encoded TableInfo."""
        return int(np.asarray(raw, dtype=np.uint8)[126]) >> 6

    def encode(self, tree_id: int, level: int, event: int, key_size: int) -> np.ndarray:
        """TreeTableInfo.encode (manifest.zig:121-149) into schema.ManifestNode.TableInfo
        (schema.zig:489-509): keys zero-padded to 32 bytes, label = level | event << 6
        (packed struct(u8) {level: u6, event: Event}, schema.zig:518-530)."""
        assert 0 < tree_id and self.value_count > 0 and 0 <= level < 64 and event in (EVENT_INSERT, EVENT_UPDATE,
                                                                                        EVENT_REMOVE)
        b = bytearray(128)
        b[0:key_size] = self.key_min.to_bytes(key_size, "little")
        b[32:32 + key_size] = self.key_max.to_bytes(key_size, "little")
        b[64:80] = self.checksum.to_bytes(16, "little")
        b[96:104] = self.address.to_bytes(8, "little")
        b[104:112] = self.snapshot_min.to_bytes(8, "little")
        b[112:120] = self.snapshot_max.to_bytes(8, "little")
        b[120:124] = self.value_count.to_bytes(4, "little")
        b[124:126] = tree_id.to_bytes(2, "little")
        b[126] = level | event << 6
        return np.frombuffer(bytes(b), dtype=np.uint8)

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
