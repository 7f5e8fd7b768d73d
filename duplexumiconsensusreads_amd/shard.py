"""Family sharding across GPUs (one process per GPU), SURVEY.md §8e.

Families (consecutive-MI runs, DuplexUMIConsensusReads.py:1209-1214) are
independent: the single-strand -> duplex dependency stays inside a family
(:1560-1582).  So the data path needs no collective:

* the host cuts the prepared family stream into CHUNKS of whole, consecutive
  families (``plan_chunks``), each of about the same cost (sum of R*L over the
  family's reads, the work the consensus kernels do);
* chunks go to ranks by greedy longest-processing-time (``assign_chunks``), so
  a few very deep families (config C4) do not pile onto one GPU;
* every rank runs its chunks through its own device (one ``dcr_run_batch`` per
  chunk) and the records come back to rank 0 tagged with their chunk number,
  where the reference's output order (:1593-1594) is restored by sorting on it
  (``gather_in_order``).

The only collectives are host-side: the object gather of finished chunks and
the small stats/timing reductions of ``bench.py`` (``max_over_ranks``,
``sum_over_ranks``).
"""
from __future__ import annotations

import heapq
from typing import List, Sequence, Tuple

from . import pipeline
from .params import ConsensusParams


def family_cost(res: pipeline.FamilyResult) -> int:
    """Work of one prepared family: bases over its (downsampled) reads."""
    if res.subs is None or res.crash is not None:
        return 0
    return sum(len(r.query_sequence or "") for sub in res.subs for r in sub)


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


def run_rank_chunks(results: List[pipeline.FamilyResult], params: ConsensusParams, backend, rank: int,
                    world: int, target_cost: int):
    """This rank's share: run every chunk it owns; returns [(chunk, results)]."""
    costs = [family_cost(r) for r in results]
    chunks = plan_chunks(costs, target_cost)
    owner = assign_chunks([sum(costs[a:b]) for a, b in chunks], world)
    done = []
    for ci, (a, b) in enumerate(chunks):
        if owner[ci] != rank:
            continue
        part = results[a:b]
        pipeline.run_batch(part, params, backend)
        done.append((ci, part))
    return done


def gather_in_order(done, group=None):
    """Host gather of finished chunks onto rank 0, reassembled in input order
    (returns the full list on rank 0, None elsewhere)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bucket = [None] * world if rank == 0 else None
    dist.gather_object(done, bucket, dst=0, group=group)
    if rank != 0:
        return None
    merged = sorted((c for per_rank in bucket for c in per_rank), key=lambda c: c[0])
    return [fam for _, part in merged for fam in part]


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
