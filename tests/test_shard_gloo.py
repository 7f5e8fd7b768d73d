"""Multi-rank family sharding (duplexumiconsensusreads_amd/shard.py) on CPU:
two `gloo` ranks each run their chunks of the small C1 BAM's families
through the C oracle backend; rank 0's gathered records must equal the
single-process run, in input order.  Also the chunk planner / LPT owner
assignment and the bench's max/sum reductions."""
import os
import random
import socket

import pytest
import torch.multiprocessing as mp

from duplexumiconsensusreads_amd import bam

from .harness import pipeline, shard
from duplexumiconsensusreads_amd.params import ConsensusParams
from tests.golden_io import GOLDEN

INPUT = os.path.join(GOLDEN, "e2e_c1_small.bam")


def prepared_families(seed=7):
    p = ConsensusParams()
    rng = random.Random(seed)
    fams, cur, code = [], None, None
    with bam.AlignmentFile(INPUT, "rb") as f:
        for r in f:
            if not (r.is_paired and r.is_proper_pair and not r.is_unmapped and not r.mate_is_unmapped
                    and not r.is_supplementary and not r.is_qcfail and r.mapping_quality >= p.min_map_quality):
                continue                                   # pass_filters (:1170-1181)
            c = r.get_tag("MI").split("/")[0]
            if cur is not None and c == code:
                cur.append(r)
            else:
                if cur is not None:
                    fams.append(cur)
                cur, code = [r], c
    fams.append(cur)
    return [pipeline.prepare_family(f, p, rng) for f in fams]


def record_dicts(results):
    return [[d.to_dict() for d in r.ds] if r.ds is not None else None for r in results]


def _worker(rank, world, port, out_path):
    import torch.distributed as dist
    from oracle import dcr_oracle_c
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = prepared_families()
        done = shard.run_rank_chunks(res, ConsensusParams(), dcr_oracle_c.run, rank, world, target_cost=9000)
        mine = sum(len(part) for _, part in done)
        merged = shard.gather_in_order(done)
        slowest = shard.max_over_ranks(float(rank + 1))
        counts = shard.sum_over_ranks([mine, 1])
        if rank == 0:
            ref = prepared_families()
            pipeline.run_batch(ref, ConsensusParams(), dcr_oracle_c.run)
            ok = (record_dicts(merged) == record_dicts(ref) and slowest == float(world)
                  and counts == [len(ref), world] and 0 < mine < len(ref))
            with open(out_path, "w") as f:
                f.write("ok" if ok else f"mismatch slowest={slowest} counts={counts} mine={mine}")
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_sharding_matches_single_process(tmp_path):
    out = tmp_path / "result.txt"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    assert out.read_text() == "ok"


def test_plan_chunks_covers_in_order():
    costs = [5, 1, 1, 9, 2, 2, 2, 0, 7]
    chunks = shard.plan_chunks(costs, 6)
    assert chunks[0][0] == 0 and chunks[-1][1] == len(costs)
    assert all(a < b for a, b in chunks)
    assert all(chunks[i][1] == chunks[i + 1][0] for i in range(len(chunks) - 1))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_lpt_balances_deep_families(world):
    # C4 shape: few loci, subfamily sizes log-uniform 100..1000 -> skewed costs
    rng = random.Random(4)
    costs = [int(150 * 4 * 10 ** rng.uniform(2, 3)) for _ in range(1000)]
    chunks = shard.plan_chunks(costs, sum(costs) // (16 * world))
    ccost = [sum(costs[a:b]) for a, b in chunks]
    owner = shard.assign_chunks(ccost, world)
    load = [0] * world
    for c, o in zip(ccost, owner):
        load[o] += c
    assert max(load) <= 1.1 * sum(load) / world
    assert shard.assign_chunks(ccost, world) == owner        # deterministic on every rank
