"""GPU parity: the HIP path (libdcr.so through its C-ABI) against the
reference's golden records and against the C oracle.  Bit-exact on every
field (bases, CIGAR, positions, MAPQ, qualities, d/e/D/M/E, statuses)."""
import random

import numpy as np
import pytest

from duplexumiconsensusreads_amd import _lib, synth
from duplexumiconsensusreads_amd.params import ConsensusParams
from oracle import dcr_oracle_c
from tests.golden_io import load_families
from tests.test_oracle_c import check_results, run_cases_with_backend

pytestmark = pytest.mark.gpu

FAM = load_families()
FIELDS = ("status", "pos", "mapq", "len", "n_cig", "n_de", "D", "M", "E")


@pytest.fixture(scope="module")
def ctx():
    c = _lib.Context(ConsensusParams(), device=0, want_info=True)
    yield c
    c.close()


def assert_same(packed, got, want):
    for kind, col_off, a, b in (("ss", packed.ss_col_off, got[0], want[0]),
                                ("ds", packed.ds_col_off, got[1], want[1])):
        for k in FIELDS:
            ga, gb = getattr(a, k), getattr(b, k)
            bad = np.nonzero(~((ga == gb) | (np.isnan(ga) & np.isnan(gb)) if ga.dtype.kind == "f" else (ga == gb)))[0]
            assert len(bad) == 0, f"{kind}.{k} differs at records {bad[:10]}: {ga[bad[:5]]} vs {gb[bad[:5]]}"
        for i in range(a.n_rec):
            if a.status[i] != 0:
                continue
            ra, rb = a.record(i, col_off), b.record(i, col_off)
            assert ra == rb, (kind, i)


@pytest.mark.parametrize("pname", sorted(FAM["params"]))
def test_gpu_matches_reference_goldens(ctx, pname):
    cases = [c for c in FAM["cases"] if c["params"] == pname]
    results, expects = run_cases_with_backend(cases, pname, _lib.backend(ctx))
    n_ok = check_results(results, expects, cases)
    assert n_ok > 0 or pname == "pre1"


def random_cfg(kind, seed):
    if kind == "C1":
        return synth.SynthConfig("t", 300, sub_size="poisson5", seed=seed)
    if kind == "indel":
        return synth.SynthConfig("t", 300, sub_size="zipf", zipf_max=40, indel_frac=0.3, seed=seed)
    if kind == "clip":
        return synth.SynthConfig("t", 300, sub_size="poisson5", indel_frac=0.1, softclip_frac=0.5, seed=seed)
    if kind == "big":
        return synth.SynthConfig("t", 6, sub_size="loguniform", logu_lo=60, logu_hi=300, indel_frac=0.05,
                                 n_loci=2, seed=seed)
    if kind == "len250":     # T around the 240/256 pairwise and LDS-scratch boundaries
        return synth.SynthConfig("t", 120, read_len=248, sub_size="poisson5", indel_frac=0.1, seed=seed)
    if kind == "len600":     # T > 256: global column scratch, deeper pairwise recursion
        return synth.SynthConfig("t", 30, read_len=600, sub_size="poisson5", indel_frac=0.2, seed=seed)
    if kind == "len90":
        return synth.SynthConfig("t", 300, read_len=90, sub_size="fixed8", seed=seed)
    if kind == "deep":       # > 64 reads per subfamily without insertions
        return synth.SynthConfig("t", 4, sub_size="loguniform", logu_lo=65, logu_hi=200, n_loci=1, seed=seed)
    return synth.SynthConfig("t", 200, sub_size="poisson5", indel_frac=0.5, softclip_frac=0.3, seed=seed)


@pytest.mark.parametrize("seed,kind", [(1, "C1"), (2, "indel"), (3, "clip"), (4, "big"), (5, "wild"),
                                       (6, "len250"), (7, "len600"), (8, "len90"), (9, "deep")])
def test_gpu_matches_oracle_random(ctx, seed, kind):
    packed = synth.packed_from_records(random_cfg(kind, seed))
    params = ConsensusParams(max_reads=10_000)
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params)
    assert_same(packed, got, want)
    for k in ("seq_start", "len", "status", "has_ins"):
        assert np.array_equal(got[2][k], want[2][k]), k


# The CLI runs without per-read info (DCR_OPT_READ_INFO off): records the
# fast kernel hands to the general kernel (invalid letters, '+' / '-' calls)
# must still see their reads' preprocessing.
@pytest.fixture(scope="module")
def ctx_noinfo():
    c = _lib.Context(ConsensusParams(), device=0, want_info=False)
    yield c
    c.close()


@pytest.mark.parametrize("pname", sorted(FAM["params"]))
def test_gpu_goldens_without_read_info(ctx_noinfo, pname):
    cases = [c for c in FAM["cases"] if c["params"] == pname]
    results, expects = run_cases_with_backend(cases, pname, _lib.backend(ctx_noinfo))
    n_ok = check_results(results, expects, cases)
    assert n_ok > 0 or pname == "pre1"


@pytest.mark.parametrize("seed,kind", [(2, "indel"), (3, "clip"), (5, "wild"), (9, "deep")])
def test_gpu_random_without_read_info(ctx_noinfo, seed, kind):
    packed = synth.packed_from_records(random_cfg(kind, seed))
    params = ConsensusParams(max_reads=10_000)
    ctx_noinfo.set_params(params)
    got = ctx_noinfo.run_host(packed, want_info=False)
    want = dcr_oracle_c.run(packed, params)
    assert_same(packed, got, want)


def test_gpu_device_path_matches_host_path(ctx):
    from duplexumiconsensusreads_amd.device import DeviceBatch
    packed = synth.packed_fixed_size(3000, seed=9)
    params = ConsensusParams()
    ctx.set_params(params)
    db = DeviceBatch(packed)
    ctx.reserve(db.batch_struct)
    ctx.run_device(db.batch_struct, db.ss_struct, db.ds_struct)
    ctx.sync()
    got = db.download()
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert_same(packed, (got[0], got[1]), want)


def test_gpu_config2_shape_properties(ctx):
    """At larger sizes: every consensus OK, duplex length == read length,
    d <= reads, e <= reads, bit-exact vs oracle on a random sample."""
    packed = synth.packed_fixed_size(20000, seed=11)
    params = ConsensusParams()
    ctx.set_params(params)
    ss, ds, _ = ctx.run_host(packed)
    assert (ss.status == 0).all() and (ds.status == 0).all()
    assert (ds.D <= 2).all() and (ss.D <= 8).all()
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert_same(packed, (ss, ds), want)


@pytest.mark.parametrize("maxq,minbq,qhi,sub", [(60, 2, 20, 3), (40, 2, 14, 8), (93, 0, 30, 8), (20, 5, 12, 2),
                                                (60, 13, 41, 8)])
def test_gpu_fast_decision_borderline(ctx, maxq, minbq, qhi, sub):
    """Low, mixed qualities put many columns within a few nats of the fast
    kernel's decision margin (ln(5 / qthresh[maxQ])): the records the fast
    kernel keeps and those it hands to the general kernel must both match the
    oracle bit for bit."""
    packed = synth.packed_fixed_size(400, sub_size=sub, read_len=150, seed=maxq + qhi)
    rng = np.random.default_rng(maxq * 7 + qhi)
    q = packed.quals
    q[:] = rng.integers(max(minbq - 1, 0), qhi + 1, q.shape, dtype=np.uint8)
    params = ConsensusParams(max_base_quality=maxq, min_base_quality=minbq)
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert_same(packed, got, want)


@pytest.mark.parametrize("maxq,minbq,qhi,sub,nfrac", [(93, 0, 93, 2, 0.05), (60, 30, 60, 2, 0.02),
                                                      (60, 13, 45, 1, 0.05), (40, 2, 40, 3, 0.1)])
def test_gpu_exact_small_records(ctx, maxq, minbq, qhi, sub, nfrac):
    """Records of one to three reads, qualities over the whole range (masked
    ones included) and sequenced 'N's: the exact pass's one-read table, its
    two-read table (single-strand pairs and every duplex record, built by
    k_r2_table at set_params) and its compacted products must match the
    oracle bit for bit."""
    packed = synth.packed_fixed_size(600, sub_size=sub, read_len=150, seed=maxq * 3 + qhi + sub)
    rng = np.random.default_rng(maxq * 11 + qhi + sub)
    q = packed.quals
    q[:] = rng.integers(0, qhi + 1, q.shape, dtype=np.uint8)
    b = packed.bases
    b[rng.random(b.shape) < nfrac] = ord("N")
    params = ConsensusParams(max_base_quality=maxq, min_base_quality=minbq)
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert_same(packed, got, want)


@pytest.mark.parametrize("config,families", [("C3", 3000), ("C4", 24), ("C5", 3000)])
def test_gpu_config_shapes_match_oracle(ctx, config, families):
    """The bench shapes of C3 (skewed sizes, indels, clips), C4 (100..1000
    reads per subfamily) and C5, from the vectorised generator the bench uses,
    bit-exact against the C oracle."""
    packed = synth.packed_config(synth.CONFIGS[config], families, seed=21, max_reads=1000)
    params = ConsensusParams(max_reads=1000)
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert_same(packed, got, want)
    for k in ("seq_start", "len", "status", "has_ins"):
        assert np.array_equal(got[2][k], want[2][k]), k


def test_gpu_deep_insertion_columns_many_classes(ctx):
    """> 64 reads with insertion columns (the general kernel's 64-read chunks)
    and error-heavy columns holding 3+ classes in several chunks: the
    per-class likelihood slots must carry across chunks."""
    cfg = synth.SynthConfig("t", 8, sub_size="loguniform", logu_lo=65, logu_hi=300, indel_frac=0.3,
                            softclip_frac=0.1, n_loci=2, seed=31)
    packed = synth.packed_config(cfg, seed=31, max_reads=1000)
    rng = np.random.default_rng(31)
    err = rng.random(packed.bases.shape) < 0.15
    packed.bases[err] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(err.sum()))]
    params = ConsensusParams(max_reads=1000, min_base_quality=10)
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert_same(packed, got, want)


@pytest.mark.parametrize("maxq,nreads", [(60, 63), (93, 63), (60, 100), (93, 130)])
def test_gpu_underflow_columns(ctx, maxq, nreads):
    """Deep high-quality columns where the reference's products underflow:
    one 'G' row beside sequenced 'N' rows at maxQ gives L = 0 for every
    class, a NaN posterior and the call 'A' (:603-618) although the LLR bound
    would decide 'G'; and a 4-way split (18/15/15/12 + 'N') at maxQ whose call
    likelihood underflows.  63 reads: the fast kernel (records above r_safe
    take the exact path); 100 / 130 reads: k_decide (its Z - L_b bound sends
    the record to the double products)."""
    L = 40
    packed = synth.packed_fixed_size(4, sub_size=nreads, read_len=L, seed=3)
    packed.quals[:] = maxq
    n_sub = len(packed.sub_off) - 1
    for s in range(n_sub):
        g0 = int(packed.sub_off[s])
        b0 = int(packed.seq_off[g0])
        tmpl = packed.bases[b0:b0 + L].copy()
        for r in range(nreads):
            o = int(packed.seq_off[g0 + r])
            packed.bases[o:o + L] = tmpl
        if s % 2 == 0:
            packed.bases[b0 + 10] = ord("G")
            for r in range(1, nreads):
                packed.bases[int(packed.seq_off[g0 + r]) + 10] = ord("N")
        else:
            col = b"G" * 18 + b"A" * 15 + b"T" * 15 + b"C" * 12 + b"N" * (nreads - 60)
            for r in range(nreads):
                packed.bases[int(packed.seq_off[g0 + r]) + 20] = col[r]
    params = ConsensusParams(max_base_quality=maxq, max_reads=1000)
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params, n_threads=8)
    assert want[0].record(0, packed.ss_col_off)["seq"][10] == "A"
    assert_same(packed, got, want)


# k_decide_deep (records of >= 64 reads): its staged codes carry the class,
# the single-strand mask and the invalid-input checks four bytes at a time,
# and its row table covers qualities 0..127.  Deep subfamilies with deletions
# and insertions, 'N', invalid letters, masked and out-of-table qualities
# sprinkled over their reads, under two mask thresholds.
@pytest.mark.parametrize("seed,minbq,rate", [(21, 20, 0.01), (22, 30, 0.02), (23, 2, 0.005)])
def test_gpu_deep_records_edge_bytes(ctx, seed, minbq, rate):
    cfg = synth.SynthConfig("t", 6, sub_size="loguniform", logu_lo=64, logu_hi=400, indel_frac=0.1,
                            softclip_frac=0.2, n_loci=1, seed=seed)
    packed = synth.packed_from_records(cfg)
    rng = np.random.default_rng(seed)
    n = len(packed.bases)
    hit = np.nonzero(rng.random(n) < rate)[0]
    kind = rng.integers(0, 4, len(hit))
    b, q = packed.bases.copy(), packed.quals.copy()
    packed.bases, packed.quals = b, q
    b[hit[kind == 0]] = ord("N")
    q[hit[kind == 1]] = 1                 # masked below min_base_quality (:280)
    q[hit[kind == 2]] = 0
    # outside the row table (the record leaves the decision pass): a few records only
    q[hit[(kind == 3) & (hit < n // 6)]] = 130
    # invalid letters (the reference exits, :580-585) in two subfamilies, one masked
    s0, s1 = packed.seq_off[packed.sub_off[5]], packed.seq_off[packed.sub_off[14]]
    b[s0 + 40] = ord("X")
    b[s1 + 7], q[s1 + 7] = ord("a"), 1
    params = ConsensusParams(max_reads=10_000, min_base_quality=minbq)
    ctx.set_params(params)
    try:
        got = ctx.run_host(packed)
        want = dcr_oracle_c.run(packed, params)
        assert_same(packed, got, want)
    finally:
        ctx.set_params(ConsensusParams())



@pytest.mark.parametrize("tail", [0, 1, 2, 3])
def test_gpu_insertion_layout_batch_end_tail(ctx, tail):
    """The batch's last record has an insertion layout whose bytes do not fit
    the stage, so its reads' next 32 bases are staged by range-checked dword
    loads; the batch's bases end `tail` bytes into a dword.  A buffer load
    returns 0 for a dword that reaches past its range, which had zeroed the
    last read's final bases (one column's depth off by one in the C3 shard,
    tools/c3shard_diff.py).  Every tail against the oracle."""
    from types import SimpleNamespace as NS

    from duplexumiconsensusreads_amd.batch import pack_families
    rng = np.random.default_rng(7 + tail)

    def read(L, cig, pos=100):
        seq = "".join("ACGT"[i] for i in rng.integers(0, 4, L))
        return NS(reference_start=pos, mapping_quality=40, query_sequence=seq,
                  query_qualities=[int(q) for q in rng.choice([37, 37, 37, 25], L)], cigartuples=cig)
    # subfamily 3 (the batch's last reads): 30 reads sharing one template, one
    # with an insertion, the last read's length setting the tail
    tmpl = "".join("ACGT"[i] for i in rng.integers(0, 4, 160))
    sub3 = []
    for j in range(30):
        L = 151 if j < 29 else 152 + tail            # 32 reads of 151 bases before it
        r = read(L, [(0, L)])
        r.query_sequence = tmpl[:L]
        sub3.append(r)
    sub3[7].cigartuples = [(0, 100), (1, 1), (0, 50)]
    fam = [[read(151, [(0, 151)])], [read(151, [(0, 151)])], [read(151, [(0, 151)])], sub3]
    packed = pack_families([fam])
    assert packed.n_bases % 4 == tail
    params = ConsensusParams()
    ctx.set_params(params)
    got = ctx.run_host(packed)
    want = dcr_oracle_c.run(packed, params)
    assert_same(packed, got, want)


def _ins_family(rng, fam):
    """a family whose four subfamilies hold insertion-heavy reads: shared and
    staggered insertions, leading insertions, deletions, soft clips, 3' N
    tails and late-starting reads (the general kernel's insertion layout by
    events, tests/fil_model.py)"""
    from tests.golden_io import input_record
    from tests.test_fil_model import _read
    L = rng.choice([24, 40, 80, 150])
    R = rng.choice([1, 2, 3, 6, 12, 30, 70])
    reads = []
    for k, (flag, strand) in enumerate(((99, "A"), (163, "B"), (83, "B"), (147, "A"))):
        for i in range(R):
            cig, b, q = _read(rng, L)
            if rng.random() < 0.3:
                a0, li = rng.randint(0, 5), rng.randint(1, 4)
                if a0 + li < L:
                    cig = ([(0, a0)] if a0 else []) + [(1, li), (0, L - a0 - li)]
            reads.append(input_record({"qname": f"f{fam}_{k}_{i}", "flag": flag, "tid": 0,
                                       "pos": 5000 + rng.randint(0, 8), "mapq": 40,
                                       "cigar": [list(x) for x in cig], "seq": b, "qual": q,
                                       "MI": f"{fam}/{strand}", "RX": "AAAA-CCCC"}))
    return reads


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_insertion_layouts_by_events(ctx, seed):
    """Insertion-heavy families through the GPU and the C oracle: every field
    of every single-strand and duplex record, and the same raising families"""
    from tests.harness import pipeline
    rng = random.Random(seed)
    fams = [_ins_family(rng, f) for f in range(400)]
    params = ConsensusParams(max_reads=10_000)
    ctx.set_params(params)
    out = []
    for backend in (_lib.backend(ctx), dcr_oracle_c.run):
        res = []
        for reads in fams:
            try:
                res.append(pipeline.prepare_family(reads, params, random.Random(0)))
            except (pipeline.FamilyExit, IndexError) as e:
                res.append(pipeline.FamilyResult(code="?", reads=reads, crash=type(e).__name__))
        pipeline.run_batch(res, params, backend)
        out.append(res)
    n = 0
    for a, b in zip(*out):
        assert a.crash == b.crash and (a.subs is None) == (b.subs is None)
        if a.crash is None and a.subs is not None:
            assert [x.to_dict() for x in a.ss] == [x.to_dict() for x in b.ss]
            assert [x.to_dict() for x in a.ds] == [x.to_dict() for x in b.ds]
            n += 1
    assert n > 100
