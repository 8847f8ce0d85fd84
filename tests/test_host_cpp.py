"""The C++ host mirror (tigerbeetle_amd/host/compaction.hpp): compiles on CPU;
its harness runs against the oracle on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "host", "compaction_host_test.cpp")
EXE = os.path.join(ROOT, "build", "compaction_host_test")


def build_harness():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = os.path.join(ROOT, "tigerbeetle_amd")
    orc = os.path.join(ROOT, "oracle")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", SRC, "-o", EXE,
                    "-L", lib, "-ltbc", "-L", orc, "-l:liboracle.so",
                    f"-Wl,-rpath,{lib}", f"-Wl,-rpath,{orc}"], check=True)
    return EXE


def test_host_mirror_compiles():
    build_harness()
    assert os.path.exists(EXE)


@pytest.mark.gpu
def test_host_mirror_against_oracle_on_gpu():
    exe = build_harness()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
