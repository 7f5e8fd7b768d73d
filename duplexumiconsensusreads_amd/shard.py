"""Family sharding helpers (one process per GPU), SURVEY.md §8e.

Families (consecutive-MI runs, DuplexUMIConsensusReads.py:1209-1214) are
independent: the single-strand -> duplex dependency stays inside a family
(:1560-1582), so the data path needs no collective.  ``bench.py`` uses these
for its device-resident lines: a shared family stream cut into chunks of about
equal cost (``plan_chunks``), dealt to ranks by greedy longest-processing-time
(``assign_chunks`` / ``rank_share``) so a few deep families (config C4) do not
pile onto one GPU; ``max_over_ranks`` / ``sum_over_ranks`` are the timing and
counter reductions.  The product CLI shards by ranges of whole families of the
input instead (cli --gpus N).
"""
from __future__ import annotations

import heapq
from typing import List, Sequence, Tuple


def plan_chunks(costs: Sequence[int], target_cost: int) -> List[Tuple[int, int]]:
    """Cut families [0, n) into consecutive chunks [a, b) of about
    ``target_cost`` each (a chunk always holds at least one family)."""
    chunks, a, acc = [], 0, 0
    for i, c in enumerate(costs):
        acc += c
        if acc >= target_cost:
            chunks.append((a, i + 1))
            a, acc = i + 1, 0
    if a < len(costs):
        chunks.append((a, len(costs)))
    return chunks


def assign_chunks(chunk_costs: Sequence[int], world: int) -> List[int]:
    """Owner rank of every chunk: greedy LPT (largest chunk first onto the
    least-loaded rank; ties go to the lower rank, so the plan is deterministic
    and identical on every rank)."""
    owner = [0] * len(chunk_costs)
    heap = [(0, r) for r in range(world)]
    for i in sorted(range(len(chunk_costs)), key=lambda i: (-chunk_costs[i], i)):
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + chunk_costs[i], r))
    return owner


def rank_share(costs: Sequence[int], rank: int, world: int, pieces_per_rank: int = 32):
    """This rank's families of one shared stream with per-family ``costs``:
    consecutive chunks of about total / (world * pieces_per_rank) each, owned
    by LPT.  Returns (increasing family indices, every rank's total cost)."""
    total = int(sum(costs))
    chunks = plan_chunks(costs, max(1, total // max(1, world * pieces_per_rank)))
    ccost = [int(sum(costs[a:b])) for a, b in chunks]
    owner = assign_chunks(ccost, world)
    loads = [0] * world
    for c, r in zip(ccost, owner):
        loads[r] += c
    mine = [f for (a, b), r in zip(chunks, owner) if r == rank for f in range(a, b)]
    return mine, loads


def max_over_ranks(x: float, device=None) -> float:
    """Max of a float over all ranks (bench timing: the slowest rank)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values: Sequence[int], device=None) -> List[int]:
    """Sum of small integer counters over all ranks (bases, bad records)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]
