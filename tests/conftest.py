import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtbc.so on the device)")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def engine():
    from tigerbeetle_amd import Engine
    e = Engine(device=0, block_size=1 << 20, profile=True)
    yield e
    e.close()


@pytest.fixture(scope="session")
def engine_small():
    """test_min-shaped engine: 4 KiB blocks (config.zig:241-269)."""
    from tigerbeetle_amd import Engine
    e = Engine(device=0, block_size=4096)
    yield e
    e.close()


@pytest.fixture(scope="session")
def engine_pipe():
    """1 MiB blocks, UNIQUE_KEYS batches always pipelined (TBC_CONFIG_PIPELINE):
    bodies merged on the engine stream, chains on a tail stream."""
    from tigerbeetle_amd import Engine
    e = Engine(device=0, block_size=1 << 20, profile=True, pipeline=True)
    yield e
    e.close()


@pytest.fixture(scope="session")
def engine_small_pipe():
    from tigerbeetle_amd import Engine
    e = Engine(device=0, block_size=4096, profile=True, pipeline=True)
    yield e
    e.close()
