"""Every environment knob libtbc.so still reads (VERDICT r4 item 7, r5 item
8) leaves the output bytes oracle-exact. The library reads them once per
process, so each setting runs, in a child process, GPU tests that exercise
the paths it changes; each of those tests compares with the oracle.

  TBC_SORT_TICKETS=1   sort passes always take tiles by ticket (the fallback
                       if the one-tile-per-workgroup path's dispatch-order
                       premise ever fails, sort.hip k_sort_pass)
  TBC_DEBUG_SYNC=1     stage-by-stage waits (tools; nothing pipelines)
  TBC_PAIR_TAILS=0     grid tails never paired (test_gpu_pairing.py)

GPU_MAX_HW_QUEUES is HIP's own (the engine sizes its tails from it). The
round-3 to round-5 A/B knobs whose paths lost every measurement (the chain
server, a sort stream of its own, tail priority, tail count, grid
speculation, job-group count, partition split threshold, drained tails on
compact tables) were removed with their paths in round 6.
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
def test_debug_sync_bit_exact():
    """TBC_DEBUG_SYNC=1 waits for every stage, so nothing pipelines: the
    parity tests that do not require it."""
    _child({"TBC_DEBUG_SYNC": "1"}, FILES, " or ".join([
        "test_compaction_parity_throughput_regime", "test_immutable_compaction_after_device_sort",
        "test_two_half_bars_chained_through_the_grid", "test_values_only_bodies_equal_full_compaction"]))


@pytest.mark.gpu
def test_sort_tickets_bit_exact():
    """TBC_SORT_TICKETS=1: every sort pass takes its tiles by ticket — the
    sort tests, the pipelined tests and the 11-bar config-1 lockstep."""
    env = {"TBC_SORT_TICKETS": "1"}
    _child(env, FILES, PIPELINED + " or test_sort_values")
    _child(env, ("test_gpu_config1.py",), "checkpoint", timeout=300)
