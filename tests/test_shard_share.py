"""Shared-stream split for the multi-GPU C4 bench (bench.shared_share):
families dealt to ranks by LPT over consecutive chunks (shard.rank_share),
each rank generating only its own families (synth.packed_config keep=)."""
import numpy as np
import pytest

from duplexumiconsensusreads_amd import batch, synth

from .harness import shard
from duplexumiconsensusreads_amd.params import ConsensusParams
from oracle import dcr_oracle_c


def _same(a, b):
    for k in batch.BATCH_FIELDS:
        x, y = getattr(a, k), getattr(b, k)
        assert x.dtype == y.dtype and np.array_equal(x, y), k


@pytest.fixture(scope="module")
def c4():
    cfg = synth.CONFIGS["C4"]
    return cfg, synth.packed_config(cfg, 40, seed=5, max_reads=1000)


def test_family_reads_match_stream(c4):
    cfg, full = c4
    reads = synth.config_family_reads(cfg, 40, seed=5, max_reads=1000)
    assert np.array_equal(reads, np.diff(full.sub_off[::4]))


def test_keep_is_subset_of_stream(c4):
    cfg, full = c4
    keep = [0, 3, 4, 5, 17, 39]
    _same(synth.packed_config(cfg, 40, seed=5, max_reads=1000, keep=keep), batch.subset_families(full, keep))


def test_subset_consensus_equals_stream(c4):
    """Consensus of a subset = the stream's consensus of those families."""
    cfg, full = c4
    keep = [1, 2, 8, 30]
    part = batch.subset_families(full, keep)
    p = ConsensusParams(max_reads=1000)
    ss_f, ds_f, _ = dcr_oracle_c.run(full, p, n_threads=4, want_info=False)
    ss_p, ds_p, _ = dcr_oracle_c.run(part, p, n_threads=4, want_info=False)
    for j, f in enumerate(keep):
        for s in range(4):
            assert ss_p.record(4 * j + s, part.ss_col_off) == ss_f.record(4 * f + s, full.ss_col_off)
        for s in range(2):
            assert ds_p.record(2 * j + s, part.ds_col_off) == ds_f.record(2 * f + s, full.ds_col_off)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rank_share_partitions_and_balances(world):
    cfg = synth.CONFIGS["C4"]
    costs = (synth.config_family_reads(cfg, 1000 * world, seed=2, max_reads=1000) * cfg.read_len).tolist()
    seen = []
    loads0 = None
    for r in range(world):
        mine, loads = shard.rank_share(costs, r, world)
        assert mine == sorted(mine)
        assert sum(costs[f] for f in mine) == loads[r]
        loads0 = loads0 or loads
        assert loads == loads0                       # the same plan on every rank
        seen += mine
    assert sorted(seen) == list(range(len(costs)))
    assert max(loads0) / (sum(loads0) / world) < 1.05


def test_bench_shared_share_two_ranks():
    import bench
    parts = [bench.shared_share("C4", 20, 2, r, 2) for r in range(2)]
    assert sum(p.n_fam for p, _ in parts) == 40
    assert parts[0][1] == parts[1][1]
    assert parts[0][1]["max_over_mean"] < 1.2
