"""TEST HARNESS: chunked multi-rank sharding of prepared families over the
pure-Python pipeline (tests/harness/pipeline.py): each rank runs the chunks
it owns (LPT over per-family cost, duplexumiconsensusreads_amd.shard) and rank
0 restores the input order (:1593-1594) from the chunk numbers."""
from __future__ import annotations

from typing import List

from duplexumiconsensusreads_amd.params import ConsensusParams
from duplexumiconsensusreads_amd.shard import (assign_chunks, max_over_ranks, plan_chunks, rank_share,  # noqa: F401
                                               sum_over_ranks)

from . import pipeline


def family_cost(res: pipeline.FamilyResult) -> int:
    """Work of one prepared family: bases over its (downsampled) reads."""
    if res.subs is None or res.crash is not None:
        return 0
    return sum(len(r.query_sequence or "") for sub in res.subs for r in sub)


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
