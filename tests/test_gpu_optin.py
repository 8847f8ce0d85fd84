"""The engine's opt-in paths, measured slower and off by default (DESIGN.md
§3), stay bit-exact: the bar-end sort on its own stream (TBC_SORT_STREAM=1:
pending-sort waits) and tails at the highest stream priority
(TBC_TAIL_PRIORITY=1). The library reads these once per process, so one
child process runs the tests that exercise those paths with both set; each
of those tests compares with the oracle."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

SELECT = " or ".join([
    "test_compaction_parity_throughput_regime",      # throughput regime: 4 pipelined groups
    "test_immutable_compaction_after_device_sort",   # sort stream, then a batch that waits on it
    "test_sort_values_batch_of_memtables",
    "test_two_half_bars_chained_through_the_grid",   # grid batches
    "test_pipelined_grid_batches_in_flight",
    "test_values_only_bodies_equal_full_compaction",  # VALUES_ONLY bodies
])


@pytest.mark.gpu
def test_opt_in_paths_bit_exact():
    env = dict(os.environ, TBC_SORT_STREAM="1", TBC_TAIL_PRIORITY="1")
    files = [os.path.join(HERE, f) for f in ("test_gpu_parity.py", "test_gpu_grid.py", "test_gpu_engine.py",
                                              "test_gpu_split.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider", "-k", SELECT,
                        *files], env=env, capture_output=True, text=True, timeout=200)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout, tail


@pytest.mark.gpu
def test_grid_speculation_bit_exact():
    """TBC_GRID_SPECULATION=1: grid batches merge their UNIQUE_KEYS jobs tile
    by tile (k_merge_unique), broken speculations recomputed in the front —
    the grid tests and the 11-bar config-1 lockstep against the oracle."""
    env = dict(os.environ, TBC_GRID_SPECULATION="1")
    files = [os.path.join(HERE, f) for f in ("test_gpu_grid.py", "test_gpu_config1.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider", *files],
                       env=env, capture_output=True, text=True, timeout=230)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout, tail
