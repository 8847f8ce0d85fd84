"""Tail pairing (engine.hip grid_tail_pair): grid batches submitted back to
back without a host wait run their chains two batches per launch. The
recording pass of config 1's replay waits for every half-bar before the
next is submitted (the Forest applies each half-bar's results first), so it
never pairs; bench.py's replay of that record submits every batch without
waiting, so consecutive half-bars pair. Replaying the record over the
recorded grid must leave every output block's header — its header and body
checksums (data_block_finish / index_block_finish, table.zig:306-457) — and
every TableInfo exactly as the unpaired recording wrote them; the recording
itself is the one test_gpu_config1.py compares with the oracle job by job.
The manifest log blocks closed on the grid while the replay's tails run
(tbc_manifest_close_blocks does not wait for them) are compared too.
"""
import numpy as np
import pytest

from tigerbeetle_amd import abi, benchmark_load

pytestmark = pytest.mark.gpu


def _headers(eng, grid, addresses):
    """The 256-byte header of every block, gathered on the device."""
    n = len(addresses)
    out = eng.alloc(256 * n)
    eng.copy_device_batch([(out.ptr + 256 * i, grid.pointer(int(a)), 256) for i, a in enumerate(addresses)])
    eng.synchronize()
    return out.download(256 * n).reshape(n, 256)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("pair", ["0", "1"])
def test_replayed_half_bars_pair_tails_bit_exact(pair, monkeypatch):
    import bench
    from tigerbeetle_amd import Engine
    monkeypatch.setenv("TBC_PAIR_TAILS", pair)  # read at engine init
    bs = 1 << 20
    bars = 38  # the whole benched replay: its checkpoint and its manifest closes included
    with Engine(device=0, block_size=bs, arena_bytes=2 << 30, profile=True) as eng:
        w = bench.ReplayWorkload(eng, bars * 32 * benchmark_load.BATCH, bs)
        comps = [c for _, hb in w.forest.history for _, c in hb if not c.move]
        addresses = sorted({int(a) for c in comps for a in c.addresses[:c.result.block_count]} |
                           {int(a) for kind, *rest in w.executor.record if kind == "manifest" for a in rest[1]})
        assert len(comps) > 100 and len(addresses) > 1000
        assert any(kind == "manifest" for kind, *_ in w.executor.record)
        before = _headers(eng, w.grid, addresses)
        # bench.ReplayWorkload.step, keeping every batch's results.
        live, paired = [], 0
        for kind, *rest in w.executor.record:
            if kind == "sort":  # from the put-order copy straight into the immutable buffer
                eng.sort_values_batch(rest[0])
            elif kind == "checkpoint":
                eng.synchronize()
            elif kind == "manifest":
                from tigerbeetle_amd import manifest
                images, addrs, prev = rest
                manifest.close_on_grid(w.grid, images, addrs, prev, None if prev else 0)
            elif kind == "batch":
                live.append((rest[0], eng.submit(rest[0])))
        infos_replay = []
        for jobs, b in live:
            b.wait()
            b.check_results()
            # The second batch of a pair marks its tail "tail_wait_paired".
            paired += "tail_wait_paired" in b.kernel_times()
            infos_replay.extend(b.result(i)[1].copy() for i in range(len(jobs)))
            b.release()
        after = _headers(eng, w.grid, addresses)
        bad = np.nonzero((before != after).any(axis=1))[0]
        if bad.size:
            owner = {}
            for bi, (jobs, _) in enumerate(live):
                for ji, job in enumerate(jobs):
                    for s, a in enumerate(job.addresses):
                        owner.setdefault(int(a), (bi, ji, s, job.tree.name))
            for i in bad[:12]:
                a = addresses[i]
                cols = np.nonzero(before[i] != after[i])[0]
                print("differs", a, owner.get(a), "bytes", cols[:8], "size", before[i][96:100].view(np.uint32),
                      after[i][96:100].view(np.uint32))
        assert bad.size == 0, f"{bad.size} of {len(addresses)} block headers differ, first at address {addresses[bad[0]]}"
        if pair == "1":
            assert paired >= len(live) // 4, (paired, len(live))
        else:
            assert paired == 0, paired
        # Every TableInfo as the recording decoded it (same jobs, same order;
        # the history holds the half-bars the forest applied, every one but
        # the last).
        from tigerbeetle_amd.forest import TableInfo
        assert len(comps) <= len(infos_replay) <= len(comps) + 64
        for c, raw in zip(comps, infos_replay):
            assert [TableInfo.decode(r, c.tree.key_size) for r in raw] == c.outputs, c.tree.name
        print(f"{len(live)} batches replayed, {paired} paired; {len(addresses)} block headers bit-exact")
