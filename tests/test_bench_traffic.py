"""bench.py's whole-step PMC traffic (roofline.traffic of a pipelined step)
read from a committed profile's traffic.json (tools/traffic.py): no alias
counted twice, warmup-only kernels left out."""
import hashlib
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from tigerbeetle_amd import abi  # noqa: E402


def test_step_traffic_skips_aliases_and_warmup_kernels(tmp_path, monkeypatch):
    lib = tmp_path / "libtbc.so"
    lib.write_bytes(b"not a library")
    md5 = hashlib.md5(lib.read_bytes()).hexdigest()
    kernels = {
        # short name = alias of the heaviest instantiation
        "k_data_blocks": {"calls": 11, "traffic_bytes": 2000},
        "k_data_blocks<false, StepBpermute>": {"calls": 11, "traffic_bytes": 2000},
        "k_data_blocks<true, StepBpermute>": {"calls": 4, "traffic_bytes": 7000},  # fused warmup steps
        "k_merge_unique": {"calls": 11, "traffic_bytes": 4000},
        "k_merge_unique<false>": {"calls": 11, "traffic_bytes": 4000},
        "k_assemble<false>": {"calls": 22, "traffic_bytes": 10},  # twice per step
        "k_index_blocks": {"calls": 15, "traffic_bytes": 3},  # every step, fused ones too
    }
    d = tmp_path / "profiles" / "rx"
    d.mkdir(parents=True)
    (d / "traffic.json").write_text(json.dumps({"lib_md5": md5, "baseline_config": 2, "kernels": kernels}))
    monkeypatch.setattr(abi, "LIB_PATH", str(lib))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    total, src = bench.pmc_step_traffic(2, "k_merge_unique")
    assert total == 2000 + 4000 + 2 * 10 + 3
    assert src == "profiles/rx/traffic.json"
    assert bench.pmc_step_traffic(3, "k_merge_unique") == (None, None)
