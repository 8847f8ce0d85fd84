"""CPU tests of the drop-in boundary: libtbc.so loads and exports every symbol
include/tbc.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os

from tigerbeetle_amd import abi


def test_library_exports_every_header_symbol():
    names = abi.header_functions()
    assert "tbc_compaction_submit" in names and "tbc_sort_values" in names
    lib = ctypes.CDLL(abi.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(abi._SIGNATURES), set(names) ^ set(abi._SIGNATURES)


def test_abi_version_and_struct_layout_match_c():
    """ctypes mirrors of the ABI structs have the C compiler's sizes/offsets."""
    import subprocess
    import tempfile
    assert abi.lib().tbc_abi_version() == abi.ABI_VERSION
    checks = {
        "tbc_tree": (abi.Tree, ["tree_id", "key_kind", "usage", "value_size", "timestamp_offset",
                                "table_value_count_max"]),
        "tbc_segment": (abi.Segment, ["values", "count"]),
        "tbc_sort_job": (abi.SortJob, ["tree", "values", "count", "values_out"]),
        "tbc_config": (abi.Config, ["device", "block_size", "arena_bytes", "flags"]),
        "tbc_compaction": (abi.Compaction, [f for f, _ in abi.Compaction._fields_ if not f.startswith("reserved")]),
        "tbc_compaction_result": (abi.CompactionResult, [f for f, _ in abi.CompactionResult._fields_]),
        "tbc_tree_layout": (abi.TreeLayout, [f for f, _ in abi.TreeLayout._fields_]),
        "tbc_table_ref": (abi.TableRef, ["address", "checksum", "value_count"]),
        "tbc_seal": (abi.Seal, [f for f, _ in abi.Seal._fields_ if not f.startswith("reserved")]),
    }
    lines = ['#include "tbc.h"', "#include <stdio.h>", "#include <stddef.h>", "int main(void) {"]
    expect = []
    for cname, (ct, fields) in checks.items():
        lines.append(f'printf("%zu\\n", sizeof({cname}));')
        expect.append(ctypes.sizeof(ct))
        for f in fields:
            lines.append(f'printf("%zu\\n", offsetof({cname}, {f}));')
            expect.append(getattr(ct, f).offset)
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(abi.HEADER_PATH), src, "-o", exe], check=True)
        got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    assert got == expect


def test_header_compiles_as_c():
    # The header is plain C (no C++ or HIP types in the signatures).
    import subprocess
    import tempfile
    src = '#include "tbc.h"\nint main(void){ tbc_engine *e = 0; (void)e; return (int)TBC_OK; }\n'
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "t.c")
        open(p, "w").write(src)
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(abi.HEADER_PATH),
                            "-c", p, "-o", os.path.join(d, "t.o")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_engine_init_without_gpu_fails_loudly():
    # No CPU fallback: without a device the engine refuses to start.
    import torch
    if torch.cuda.is_available():
        return
    cfg = abi.Config(0, 1 << 20, 0, 0, 0)
    h = ctypes.c_void_p()
    assert abi.lib().tbc_engine_init(ctypes.byref(cfg), ctypes.byref(h)) == abi.TBC_ERR_DEVICE
