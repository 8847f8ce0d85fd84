"""ctypes binding of the C ABI in include/tbc.h (libtbc.so).

The library is built in-tree (tigerbeetle_amd/libtbc.so) by `make -C
tigerbeetle_amd/csrc` or `__graft_entry__.build()`. There is no CPU fallback:
if the library (or a GPU) is missing, calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TBC_LIB") or os.path.join(HERE, "libtbc.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "tbc.h")

TBC_OK = 0
TBC_PENDING = 1
TBC_ERR_INVALID_ARGUMENT = 2
TBC_ERR_DEVICE = 3
TBC_ERR_OUT_OF_MEMORY = 4
TBC_ERR_CAPACITY = 5
TBC_ERR_INVARIANT = 6
TBC_ERR_BLOCK_INVALID = 7
STATUS_NAMES = {
    0: "OK", 1: "PENDING", 2: "ERR_INVALID_ARGUMENT", 3: "ERR_DEVICE", 4: "ERR_OUT_OF_MEMORY",
    5: "ERR_CAPACITY", 6: "ERR_INVARIANT", 7: "ERR_BLOCK_INVALID",
}

KEY_TIMESTAMP, KEY_ID_U128, KEY_COMPOSITE_U64, KEY_COMPOSITE_U128 = 0, 1, 2, 3
USAGE_GENERAL, USAGE_SECONDARY_INDEX = 0, 1
CONFIG_PROFILE = 1
CONFIG_PIPELINE = 2
CONFIG_LATENCY = 4
COMPACTION_VALUES_ONLY = 1  # tbc_compaction.flags
COMPACTION_GRID = 2
COMPACTION_UNIQUE_KEYS = 4  # speculated merge (tbc.h): no repeated key in A u B, no tombstone dropped
COMPACTION_COUNT_ONLY = 8  # the merge alone: survivor counts (phase A of a split job)
SPECULATION_NONE, SPECULATION_HELD, SPECULATION_BROKEN = 0, 1, 2
ABI_VERSION = 7


class TbcError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {STATUS_NAMES.get(status, status)}")
        self.status = status


class Tree(ctypes.Structure):
    _fields_ = [
        ("tree_id", ctypes.c_uint16),
        ("key_kind", ctypes.c_uint8),
        ("usage", ctypes.c_uint8),
        ("value_size", ctypes.c_uint32),
        ("timestamp_offset", ctypes.c_uint32),
        ("table_value_count_max", ctypes.c_uint32),
    ]


class TreeLayout(ctypes.Structure):
    _fields_ = [
        ("key_size", ctypes.c_uint32),
        ("block_value_count_max", ctypes.c_uint32),
        ("data_block_count_max", ctypes.c_uint32),
        ("index_size", ctypes.c_uint32),
        ("index_checksums_offset", ctypes.c_uint32),
        ("index_keys_min_offset", ctypes.c_uint32),
        ("index_keys_max_offset", ctypes.c_uint32),
        ("index_addresses_offset", ctypes.c_uint32),
    ]


class Config(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("block_size", ctypes.c_uint32),
        ("arena_bytes", ctypes.c_uint64),
        ("flags", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


class Segment(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("count", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class SortJob(ctypes.Structure):
    _fields_ = [("tree", Tree), ("values", ctypes.c_void_p), ("count", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("values_out", ctypes.c_void_p)]


class Copy(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_void_p), ("src", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


class TableRef(ctypes.Structure):
    _fields_ = [("address", ctypes.c_uint64), ("checksum", ctypes.c_uint64 * 2), ("value_count", ctypes.c_uint64)]


class Compaction(ctypes.Structure):
    _fields_ = [
        ("tree", Tree),
        ("a_immutable", ctypes.c_uint8),
        ("drop_tombstones", ctypes.c_uint8),
        ("level_b", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
        ("reserved1", ctypes.c_uint32),
        ("segments_a", ctypes.POINTER(Segment)),
        ("segment_count_a", ctypes.c_uint32),
        ("segment_count_b", ctypes.c_uint32),
        ("segments_b", ctypes.POINTER(Segment)),
        ("cluster", ctypes.c_uint64 * 2),
        ("snapshot_min", ctypes.c_uint64),
        ("addresses", ctypes.POINTER(ctypes.c_uint64)),
        ("address_count", ctypes.c_uint32),
        ("reserved2", ctypes.c_uint32),
        ("output_blocks", ctypes.c_void_p),
        ("grid", ctypes.c_void_p),
        ("tables_a", ctypes.POINTER(TableRef)),
        ("tables_b", ctypes.POINTER(TableRef)),
        ("table_count_a", ctypes.c_uint32),
        ("table_count_b", ctypes.c_uint32),
        ("output_offset", ctypes.c_uint64),
    ]


class Seal(ctypes.Structure):
    """tbc_seal: sealing of one job split by key range (tbc_compaction_seal)."""
    _fields_ = [
        ("tree", Tree),
        ("cluster", ctypes.c_uint64 * 2),
        ("snapshot_min", ctypes.c_uint64),
        ("level_b", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 3),
        ("address_count", ctypes.c_uint32),
        ("addresses", ctypes.POINTER(ctypes.c_uint64)),
        ("output_blocks", ctypes.c_void_p),
        ("value_count", ctypes.c_uint64),
        ("block_first", ctypes.c_uint32),
        ("block_count", ctypes.c_uint32),
        ("table_first", ctypes.c_uint32),
        ("table_count", ctypes.c_uint32),
    ]


class CompactionResult(ctypes.Structure):
    _fields_ = [
        ("value_count", ctypes.c_uint64),
        ("data_block_count", ctypes.c_uint32),
        ("table_count", ctypes.c_uint32),
        ("block_count", ctypes.c_uint32),
        ("status", ctypes.c_uint32),
    ]


# Every function include/tbc.h declares, with its ctypes signature.
_P = ctypes.c_void_p
_SIGNATURES = {
    "tbc_abi_version": (ctypes.c_uint32, []),
    "tbc_engine_init": (ctypes.c_int, [ctypes.POINTER(Config), ctypes.POINTER(_P)]),
    "tbc_engine_deinit": (None, [_P]),
    "tbc_tree_layout_get": (ctypes.c_int, [_P, ctypes.POINTER(Tree), ctypes.POINTER(TreeLayout)]),
    "tbc_engine_arena_usage": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                              ctypes.POINTER(ctypes.c_uint32)]),
    "tbc_host_register": (ctypes.c_int, [_P, _P, ctypes.c_uint64]),
    "tbc_host_unregister": (ctypes.c_int, [_P, _P]),
    "tbc_device_alloc": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.POINTER(_P)]),
    "tbc_device_free": (ctypes.c_int, [_P, _P]),
    "tbc_copy_to_device": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64]),
    "tbc_copy_to_host": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64]),
    "tbc_memset_device": (ctypes.c_int, [_P, _P, ctypes.c_int, ctypes.c_uint64]),
    "tbc_synchronize": (ctypes.c_int, [_P]),
    "tbc_checksum_batch": (ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.c_uint32, _P]),
    "tbc_copy_device_async": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64]),
    "tbc_copy_device_batch": (ctypes.c_int, [_P, ctypes.POINTER(Copy), ctypes.c_uint32]),
    "tbc_blocks_validate": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_uint32, _P]),
    "tbc_sort_values": (ctypes.c_int, [_P, ctypes.POINTER(Tree), _P, ctypes.c_uint32]),
    "tbc_sort_values_async": (ctypes.c_int, [_P, ctypes.POINTER(Tree), _P, ctypes.c_uint32]),
    "tbc_sort_values_batch": (ctypes.c_int, [_P, ctypes.POINTER(SortJob), ctypes.c_uint32]),
    "tbc_kway_merge": (ctypes.c_int, [_P, ctypes.POINTER(Tree), ctypes.POINTER(Segment), ctypes.c_uint32,
                                      ctypes.c_uint32, _P, ctypes.POINTER(ctypes.c_uint64)]),
    "tbc_kway_merge_submit": (ctypes.c_int, [_P, ctypes.POINTER(Tree), ctypes.POINTER(Segment), ctypes.c_uint32,
                                             ctypes.c_uint32, _P, ctypes.POINTER(_P)]),
    "tbc_kway_poll": (ctypes.c_int, [_P]),
    "tbc_kway_wait": (ctypes.c_int, [_P]),
    "tbc_kway_count": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "tbc_kway_release": (None, [_P]),
    "tbc_compaction_seal": (ctypes.c_int, [_P, ctypes.POINTER(Seal), ctypes.POINTER(_P)]),
    "tbc_compaction_submit": (ctypes.c_int, [_P, ctypes.POINTER(Compaction), ctypes.c_uint32,
                                             ctypes.POINTER(_P)]),
    "tbc_batch_poll": (ctypes.c_int, [_P]),
    "tbc_batch_wait": (ctypes.c_int, [_P]),
    "tbc_batch_result": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.POINTER(CompactionResult), _P,
                                        ctypes.c_uint32]),
    "tbc_batch_speculation": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    "tbc_batch_kernel_times": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_char_p),
                                              ctypes.POINTER(ctypes.c_double), ctypes.c_uint32,
                                              ctypes.POINTER(ctypes.c_uint32)]),
    "tbc_batch_release": (None, [_P]),
    "tbc_grid_init": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.POINTER(_P)]),
    "tbc_grid_deinit": (None, [_P]),
    "tbc_grid_block_pointer": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.POINTER(_P)]),
    "tbc_grid_put_blocks": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_P), ctypes.c_uint32]),
    "tbc_grid_invalidate": (ctypes.c_int, [_P]),
    "tbc_grid_get_blocks": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_P), ctypes.c_uint32]),
    "tbc_manifest_close_blocks": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_P),
                                                 ctypes.c_uint32, ctypes.c_uint64, _P]),
    "tbc_manifest_close_status": (ctypes.c_int, [_P]),
    "tbc_memtable_init": (ctypes.c_int, [_P, ctypes.POINTER(Tree), ctypes.c_uint32, ctypes.POINTER(_P)]),
    "tbc_memtable_deinit": (None, [_P]),
    "tbc_memtable_put": (ctypes.c_int, [_P, _P, ctypes.c_uint32]),
    "tbc_memtable_values": (ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_uint32)]),
    "tbc_memtable_reset": (ctypes.c_int, [_P]),
    "tbc_engine_stream": (ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    "tbc_engine_set_profile": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "tbc_memtable_make_immutable": (ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P), _P, ctypes.c_uint32]),
}

_lib = None


def header_functions() -> list[str]:
    """Function names declared in include/tbc.h."""
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(tbc_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load libtbc.so (raises if it was not built: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C tigerbeetle_amd/csrc` "
                               "or __graft_entry__.build(); there is no CPU fallback")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def check(status: int, what: str) -> None:
    if status != TBC_OK:
        raise TbcError(status, what)
