"""Every environment knob libtbc.so still reads leaves
the output bytes oracle-exact. The library reads them once per process, so
each setting runs, in a child process, GPU tests that exercise the paths it
changes; each of those tests compares with the oracle.

  TBC_SORT_STREAM=1, TBC_TAIL_PRIORITY=1   bar-end sorts on their own stream
                                           (pending-sort waits), tails at the
                                           highest stream priority
  TBC_GRID_SPECULATION=1                   grid batches merge UNIQUE_KEYS jobs
                                           tile by tile, recompute in front
  TBC_TAILS=2                              two tail streams
  TBC_DEBUG_SYNC=1                         stage-by-stage waits (nothing pipelines)
  TBC_PAIR_TAILS=0                         grid tails never paired (test_gpu_pairing.py)
  TBC_CHAIN_SERVER=1                       the chain server (round 5, opt-in):
                                           every batch's chains claimed by one
                                           server on its own stream
  TBC_CHAIN_SERVER=1, TBC_SERVER_WGS=64,   a small server whose idle waves
  TBC_SERVER_WAVES=4,                      leave at once and poll slowly; two
  TBC_CHAIN_LINGER_US=0,                   job groups in the throughput regime
  TBC_CHAIN_BACKOFF=128, TBC_GROUPS=2
  TBC_SORT_TICKETS=1, TBC_WAVE_SPLITS=4096,  sort passes take tiles by ticket,
  TBC_DRAIN_COMPACT=1                      mask-merge partitions by thread above
                                           4,096 splits, drained grid tails on
                                           the compact tables (round 5 A/B)

GPU_MAX_HW_QUEUES is HIP's own (the engine sizes its tails from it).
"""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

# Pipelined, grid and throughput-regime batches, sorts, overlapping tails.
PIPELINED = " or ".join([
    "test_compaction_parity_throughput_regime",      # throughput regime: pipelined job groups
    "test_immutable_compaction_after_device_sort",   # a batch after a device sort
    "test_sort_values_batch_of_memtables",
    "test_two_half_bars_chained_through_the_grid",   # grid batches
    "test_pipelined_grid_batches_in_flight",
    "test_values_only_bodies_equal_full_compaction",  # VALUES_ONLY bodies
    "test_speculated_batches_pipelined_three_in_flight",
    "test_back_to_back_batches_share_outputs",
])
FILES = ("test_gpu_parity.py", "test_gpu_grid.py", "test_gpu_engine.py", "test_gpu_split.py", "test_gpu_overlap.py")


def _child(env_extra: dict, files, select=None, timeout=240):
    env = dict(os.environ, **env_extra)
    args = [sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider"]
    if select:
        args += ["-k", select]
    r = subprocess.run(args + [os.path.join(HERE, f) for f in files], env=env, capture_output=True, text=True,
                       timeout=timeout)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout, tail


@pytest.mark.gpu
def test_sort_stream_and_tail_priority_bit_exact():
    _child({"TBC_SORT_STREAM": "1", "TBC_TAIL_PRIORITY": "1"}, FILES, PIPELINED)


@pytest.mark.gpu
def test_grid_speculation_bit_exact():
    """TBC_GRID_SPECULATION=1: grid batches merge their UNIQUE_KEYS jobs tile
    by tile (k_merge_unique), broken speculations recomputed in the front —
    the grid tests and the 11-bar config-1 lockstep against the oracle."""
    _child({"TBC_GRID_SPECULATION": "1"}, ("test_gpu_grid.py", "test_gpu_config1.py"), timeout=300)


@pytest.mark.gpu
def test_two_tails_bit_exact():
    _child({"TBC_TAILS": "2"}, FILES, PIPELINED)


@pytest.mark.gpu
def test_debug_sync_bit_exact():
    """TBC_DEBUG_SYNC=1 waits for every stage, so nothing pipelines: the
    parity tests that do not require it."""
    _child({"TBC_DEBUG_SYNC": "1"}, FILES, " or ".join([
        "test_compaction_parity_throughput_regime", "test_immutable_compaction_after_device_sort",
        "test_two_half_bars_chained_through_the_grid", "test_values_only_bodies_equal_full_compaction"]))


@pytest.mark.gpu
def test_chain_server_bit_exact():
    """The chain server with its default geometry: the pipelined, grid and
    throughput-regime tests, and the 11-bar config-1 lockstep with a
    checkpoint and restart."""
    _child({"TBC_CHAIN_SERVER": "1"}, FILES, PIPELINED)
    _child({"TBC_CHAIN_SERVER": "1"}, ("test_gpu_config1.py",), "checkpoint", timeout=300)


@pytest.mark.gpu
def test_small_chain_server_bit_exact():
    _child({"TBC_CHAIN_SERVER": "1", "TBC_SERVER_WGS": "64", "TBC_SERVER_WAVES": "4", "TBC_CHAIN_LINGER_US": "0",
            "TBC_CHAIN_BACKOFF": "128", "TBC_GROUPS": "2"}, FILES, PIPELINED)


@pytest.mark.gpu
def test_round5_ab_knobs_bit_exact():
    """The round-5 A/B knobs restore the earlier paths: the sort and grid
    tests (tickets in every pass, thread partitions, compact drained tails)
    and the 11-bar config-1 lockstep."""
    env = {"TBC_SORT_TICKETS": "1", "TBC_WAVE_SPLITS": "4096", "TBC_DRAIN_COMPACT": "1"}
    _child(env, FILES, PIPELINED + " or test_sort_values")
    _child(env, ("test_gpu_config1.py",), "checkpoint", timeout=300)
