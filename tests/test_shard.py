"""Multi-GPU path on CPU: the shard plan and the max-over-ranks reduction,
with world_size 2 over gloo (the GPU runs use RCCL; the logic is identical)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tigerbeetle_amd.shard import plan_shards, reduce_step


def test_plan_is_a_balanced_partition():
    sizes = [75, 75, 75, 12, 40, 8, 33, 75, 1, 64]
    for world in (1, 2, 4, 8):
        plan = plan_shards(sizes, world)
        flat = sorted(i for p in plan for i in p)
        assert flat == list(range(len(sizes)))
        loads = [sum(sizes[i] for i in p) for p in plan]
        assert max(loads) - min(loads) <= max(sizes)
    # weak scaling: 28 equal jobs per GPU
    plan = plan_shards([1] * 28 * 8, 8)
    assert all(len(p) == 28 for p in plan)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sizes = [100 + 7 * i for i in range(12)]
    plan = plan_shards(sizes, world)          # identical on every rank
    mine = plan[rank]
    local_bytes = sum(sizes[i] for i in mine)
    local_seconds = 1.0 + rank                # rank 1 is slower
    total, t = reduce_step(dist, local_bytes, local_seconds)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    q.put((rank, total, t, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_reduction_over_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [100 + 7 * i for i in range(12)]
    for rank, total, t, gathered in out:
        assert total == sum(sizes)            # every job counted exactly once
        assert t == 2.0                       # max over ranks
        assert sorted(i for g in gathered for i in g) == list(range(12))


def test_forest_plan_balances_bytes():
    # Config 4: jobs of 4 key kinds and 3 sizes; every rank's load stays within
    # one job of the mean (LPT), for every world size the bench runs.
    from tigerbeetle_amd import configs
    for world in (1, 2, 4, 8):
        sizes = [configs.job_bytes(4, j) for j in range(configs.FOREST_JOBS * world)]
        plan = plan_shards(sizes, world)
        assert sorted(i for p in plan for i in p) == list(range(len(sizes)))
        loads = [sum(sizes[i] for i in p) for p in plan]
        assert max(loads) - min(loads) <= max(sizes)
