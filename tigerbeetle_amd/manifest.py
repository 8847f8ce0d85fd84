"""Manifest-log blocks from a compaction's TableInfos.

The reference appends each output table's `ManifestNode.TableInfo` to the
manifest log (`Manifest.insert_table`, manifest.zig:233-255 →
`ManifestLog.append`), which packs them into manifest blocks of at most
`entry_count_max = (block_size − 256) / 128` entries
(schema.zig:451-595) and closes each block (manifest_log.zig:876-952):

  header: cluster, address (grid.acquire), snapshot 0, command block,
          block_type manifest (3), size = 256 + 128·entry_count,
          metadata = {previous block's checksum, 0, previous block's address,
          entry_count, 52 zero bytes}; checksum_body, then checksum.

Each block links to the previous one by its header checksum, so headers are a
chain; bodies are independent. Here the bodies of all blocks are checksummed
in ONE GPU batch (`tbc_checksum_batch`, up to 1 MiB each), then the 240-byte
header checksums follow the chain on the GPU, one per block. Packing the
bytes is host work, as in the reference.
"""
from __future__ import annotations

import numpy as np

from .trees import HEADER_SIZE, SECTOR_SIZE

TABLE_INFO_SIZE = 128
BLOCK_TYPE_MANIFEST = 3   # schema.zig:57-65
COMMAND_BLOCK = 20        # vsr.zig:196


def entry_count_max(block_size: int) -> int:
    return (block_size - HEADER_SIZE) // TABLE_INFO_SIZE


def pack_blocks(table_infos: np.ndarray, addresses, cluster: int, block_size: int,
                previous_address: int = 0) -> list:
    """Headers (checksums and previous-checksum links still zero) and bodies of
    the manifest blocks holding `table_infos` in order, one per address."""
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


def manifest_blocks(engine, table_infos: np.ndarray, addresses, cluster: int, previous_checksum: int = 0,
                    previous_address: int = 0):
    """Close the manifest blocks of `table_infos` (manifest_log.zig:876-952)
    with GPU checksums. Returns (disk images, header checksums)."""
    bs = engine.block_size
    blocks = pack_blocks(table_infos, addresses, cluster, bs, previous_address)
    if not blocks:
        return [], []
    if len(addresses) < len(blocks):
        raise ValueError("one address per manifest block")
    sizes = [int(b[96:100].view(np.uint32)[0]) for b in blocks]
    dev = [engine.upload(b) for b in blocks]
    body = engine.checksum_device([d.ptr + HEADER_SIZE for d in dev], [s - HEADER_SIZE for s in sizes])
    prev = int(previous_checksum)
    sums = []
    for b, d, bsum in zip(blocks, dev, body):
        b[32:48] = bsum                                    # set_checksum_body
        b[128:144] = np.frombuffer(prev.to_bytes(16, "little"), np.uint8)
        d.upload(b[:HEADER_SIZE])
        hsum = engine.checksum_device([d.ptr + 16], [HEADER_SIZE - 16])[0]
        b[0:16] = hsum                                     # set_checksum
        prev = int.from_bytes(hsum.tobytes(), "little")
        sums.append(prev)
    return blocks, sums
