"""GPU parity at bench scale: the device path the bench times
(``DeviceBatch`` + ``dcr_run_batch``, inputs resident in HBM) on full-size
batches of every BASELINE.json shape, compared field by field with the C
oracle (oracle/dcr_oracle.c, 16 threads) on the same inputs.

* C2: the whole 312,500-family bench batch (10 M reads);
* C3: a 100,000-family shard (Zipf sizes, indels, clips) - the persistent
  general kernel and k_decide over a shard of ~3 M reads;
* C4: 1,000 families of 100..1,000 reads per subfamily (``--max_reads 1000``);
* C5: one 4 M-read streaming chunk (Poisson(4)+1 subfamilies).

Comparisons are vectorised: every scalar field of every record, and the
variable-length fields (seq, qual, cigar, d, e) over each OK record's filled
part of its region.  Per-read preprocessing info is compared for every read.
"""
import numpy as np
import pytest

from duplexumiconsensusreads_amd import _lib, synth
from duplexumiconsensusreads_amd.params import ConsensusParams
from oracle import dcr_oracle_c

pytestmark = pytest.mark.gpu

SCALARS = ("status", "pos", "mapq", "len", "n_cig", "n_de", "D", "M", "E")
VARLEN = (("seq", "len"), ("qual", "len"), ("cigar", "n_cig"), ("d", "n_de"), ("e", "n_de"))


def region_index(off, n):
    """Flat indices of the ranges [off[i], off[i] + n[i])."""
    n = n.astype(np.int64)
    if n.sum() == 0:
        return np.zeros(0, np.int64)
    first = np.concatenate([[0], np.cumsum(n)[:-1]])
    return np.repeat(off.astype(np.int64) - first, n) + np.arange(int(n.sum()), dtype=np.int64)


def assert_same_kind(kind, col_off, a, b):
    for k in SCALARS:
        ga, gb = getattr(a, k), getattr(b, k)
        same = (ga == gb) | (np.isnan(ga) & np.isnan(gb)) if ga.dtype.kind == "f" else (ga == gb)
        bad = np.nonzero(~same)[0]
        assert len(bad) == 0, f"{kind}.{k} differs at {len(bad)} records, first {bad[:8]}: {ga[bad[:4]]} vs {gb[bad[:4]]}"
    ok = a.status == 0
    off = np.asarray(col_off[:-1])[ok]
    for field, nf in VARLEN:
        idx = region_index(off, getattr(a, nf)[ok])
        ga, gb = getattr(a, field)[idx], getattr(b, field)[idx]
        bad = np.nonzero(ga != gb)[0]
        assert len(bad) == 0, f"{kind}.{field} differs at {len(bad)} columns, first flat index {idx[bad[:4]]}"


def run_device_vs_oracle(ctx, packed, params):
    from duplexumiconsensusreads_amd.device import DeviceBatch
    ctx.set_params(params)
    db = DeviceBatch(packed)
    ctx.reserve(db.batch_struct)
    ctx.run_device(db.batch_struct, db.ss_struct, db.ds_struct)
    ctx.sync()
    ss, ds = db.download()
    info = ctx.read_info(packed.n_reads) if ctx.want_info else None
    del db
    want_ss, want_ds, want_info = dcr_oracle_c.run(packed, params, n_threads=16)
    assert_same_kind("ss", packed.ss_col_off, ss, want_ss)
    assert_same_kind("ds", packed.ds_col_off, ds, want_ds)
    if info is not None:
        for k in ("seq_start", "len", "status", "has_ins"):
            bad = np.nonzero(info[k] != want_info[k])[0]
            assert len(bad) == 0, f"read info {k} differs at {len(bad)} reads, first {bad[:8]}"
    return ss, ds


@pytest.fixture(scope="module")
def ctx():
    # the bench's configuration: per-read info only for failing reads
    c = _lib.Context(ConsensusParams(), device=0)
    c.want_info = False
    yield c
    c.close()


@pytest.fixture(scope="module")
def ctx_info():
    c = _lib.Context(ConsensusParams(), device=0, want_info=True)
    c.want_info = True
    yield c
    c.close()


def test_gpu_scale_c2_full_bench_batch(ctx):
    packed = synth.packed_fixed_size(312_500, seed=2)
    ss, ds = run_device_vs_oracle(ctx, packed, ConsensusParams())
    assert (ss.status == 0).all() and (ds.status == 0).all()


@pytest.mark.parametrize("config,families", [("C3", 100_000), ("C4", 1_000), ("C5", 200_000)])
def test_gpu_scale_config_shards(ctx, config, families):
    packed = synth.packed_config(synth.CONFIGS[config], families, seed=23, max_reads=1000)
    run_device_vs_oracle(ctx, packed, ConsensusParams(max_reads=1000))


def test_gpu_scale_c3_read_info(ctx_info):
    """With DCR_OPT_READ_INFO every read's preprocessing info matches too."""
    packed = synth.packed_config(synth.CONFIGS["C3"], 30_000, seed=29, max_reads=1000)
    run_device_vs_oracle(ctx_info, packed, ConsensusParams(max_reads=1000))
