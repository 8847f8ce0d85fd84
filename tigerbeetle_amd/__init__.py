"""tigerbeetle_amd — MI355X-native LSM compaction engine for TigerBeetle's forest.

The product is libtbc.so (HIP kernels for gfx950 behind the C ABI in
include/tbc.h). This package is the host-side plumbing over that ABI
(ctypes), the forest's tree table parameters and synthetic workloads.
"""
from . import abi, trees  # noqa: F401
from .engine import Batch, DeviceBuffer, Engine, Grid, Job, Memtable, stage_blocks  # noqa: F401

__all__ = ["abi", "trees", "Engine", "Grid", "Job", "Memtable", "Batch", "DeviceBuffer", "stage_blocks"]
