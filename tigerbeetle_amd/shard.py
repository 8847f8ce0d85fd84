"""Multi-GPU sharding of a half-bar's compactions.

Every (tree, level) compaction of a half-bar is independent: disjoint trees
and disjoint grid reservations (compaction.zig:312-318, free_set.zig:240-345).
So jobs shard across GPUs with no data-path collective — each rank runs its
own batch on its own GPU (one process per GPU) — and the only communication
is the timing/metrics reduction. Assignment is greedy longest-processing-time
by input bytes (a job's time is proportional to its bytes).
"""
from __future__ import annotations


def plan_shards(job_bytes: list, world: int) -> list:
    """Partition job indices over `world` ranks, balancing total bytes (LPT).
    Deterministic: every rank computes the same plan without communicating."""
    assert world >= 1
    order = sorted(range(len(job_bytes)), key=lambda i: (-job_bytes[i], i))
    loads = [0] * world
    plan = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (loads[k], k))
        plan[r].append(i)
        loads[r] += job_bytes[i]
    for p in plan:
        p.sort()
    return plan


def reduce_step(dist, local_bytes: int, local_seconds: float, device=None):
    """Whole-job aggregate over ranks: (sum of bytes, max of seconds)."""
    if dist is None:
        return local_bytes, local_seconds
    import torch
    t = torch.tensor([local_seconds], dtype=torch.float64, device=device)
    b = torch.tensor([float(local_bytes)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return int(b.item()), float(t.item())
