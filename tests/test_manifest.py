"""Manifest-log blocks: the oracle restatement of
ManifestLog.close_block (manifest_log.zig:876-952) checked against the
reference's structural asserts (schema.zig:534-554 ManifestNode.metadata,
:574-580 size, manifest_log.zig:954-960 verify_block) and the chain links;
the GPU path (tigerbeetle_amd/manifest.py) must equal it byte for byte."""
import numpy as np
import pytest

from oracle import oracle
from tigerbeetle_amd import manifest

CLUSTER = 0xA1B2C3D4E5F60718293A4B5C6D7E8F90


def _infos(n, seed=0):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(n, 128), dtype=np.uint8)


@pytest.mark.parametrize("bs,n", [(4096, 1), (4096, 30), (4096, 31), (4096, 95), (1 << 20, 8190), (1 << 20, 9000)])
def test_oracle_manifest_blocks_structure(bs, n):
    addrs = list(range(500, 600, 7))
    imgs, sums = oracle.manifest_blocks(_infos(n), addrs, CLUSTER, bs, previous_checksum=0x55, previous_address=9)
    m = (bs - 256) // 128
    assert len(imgs) == -(-n // m)
    for b, (img, c) in enumerate(zip(imgs, sums)):
        size = int(img[96:100].view(np.uint32)[0])
        count = int(img[168:172].view(np.uint32)[0])
        assert 0 < count <= m and count == (size - 256) // 128            # schema.zig:542-545
        assert not img[144:160].any() and not img[172:224].any()          # padding, reserved (:546-547)
        assert int(img[232:240].view(np.uint64)[0]) == 0 and img[240] == 3 and img[110] == 20
        assert int(img[224:232].view(np.uint64)[0]) == addrs[b]
        prev_a = int(img[160:168].view(np.uint64)[0])
        prev_c = int.from_bytes(img[128:144].tobytes(), "little")
        assert (prev_a, prev_c) == ((9, 0x55) if b == 0 else (addrs[b - 1], sums[b - 1]))
        assert not img[size:].any()                                        # zero padding (:931-932)
        assert oracle.checksum(img[256:size].tobytes()) == int.from_bytes(img[32:48].tobytes(), "little")
        assert oracle.checksum(img[16:256].tobytes()) == c == int.from_bytes(img[0:16].tobytes(), "little")
        assert np.array_equal(img[256:size].reshape(-1, 128), _infos(n)[b * m:b * m + count])


def test_pack_matches_oracle_layout():
    # host packing of the product path = the oracle's bytes before checksums
    infos = _infos(70, 3)
    imgs, _ = oracle.manifest_blocks(infos, [11, 12, 13], CLUSTER, 4096, previous_address=4)
    packed = manifest.pack_blocks(infos, [11, 12, 13], CLUSTER, 4096, previous_address=4)
    assert len(packed) == len(imgs)
    for p, o in zip(packed, imgs):
        q = o.copy()
        q[0:16] = 0
        q[32:48] = 0
        q[128:144] = 0
        assert np.array_equal(p, q)


@pytest.mark.gpu
@pytest.mark.parametrize("bs,n", [(4096, 1), (4096, 95), (1 << 20, 1000), (1 << 20, 20000)])
def test_gpu_manifest_blocks_equal_oracle(bs, n):
    from tigerbeetle_amd import Engine
    addrs = list(range(1000, 1010))
    with Engine(device=0, block_size=bs) as eng:
        got, gsums = manifest.manifest_blocks(eng, _infos(n, n), addrs, CLUSTER, previous_checksum=7,
                                              previous_address=3)
    want, wsums = oracle.manifest_blocks(_infos(n, n), addrs, CLUSTER, bs, previous_checksum=7, previous_address=3)
    assert gsums == wsums
    assert all(np.array_equal(g, w) for g, w in zip(got, want)) and len(got) == len(want)


def test_no_entries_no_blocks():
    # close_block asserts entry_count > 0 (manifest_log.zig:913): nothing to close
    assert manifest.pack_blocks(np.zeros((0, 128), np.uint8), [], CLUSTER, 4096) == []
    assert oracle.manifest_blocks(np.zeros((0, 128), np.uint8), [], CLUSTER, 4096) == ([], [])
