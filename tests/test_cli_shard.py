"""Sharded CLI (``--gpus N``: one process per GPU over ranges of whole
families, cli._main_sharded) against the single-process CLI on the same
input: 2 and 3 gloo ranks on CPU, the C oracle as the batch backend (test
infrastructure; the ranks' GPU path is the same code with the HIP backend).

Identical means: the three output BAMs record for record, stdout, the
exception, and the caller's random state afterwards.  Cases: excluded reads
and filtered families; downsampling in every range (the ranks' random
states come from the calls of the ranks before them: each later
rank's ingest waits at its first random.sample call for the state after the
earlier ranks' calls, which those ranks publish from their own pass or from a
host-only count pass; no rank runs twice); the reference stopping at a read
inside the first or the second range, with and without downsampling."""
import contextlib
import io
import multiprocessing as mp
import os
import random
import socket

import pytest

from duplexumiconsensusreads_amd import bam, cli, native_io, synth
from duplexumiconsensusreads_amd.params import ConsensusParams
from oracle import dcr_oracle_c


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _outcome(argv, seed, stats=None):
    rng = random.Random(seed)
    buf = io.StringIO()
    exc = None
    try:
        with contextlib.redirect_stdout(buf):
            cli.main(argv, backend=dcr_oracle_c.run, rng=rng, stats=stats)
    except SystemExit as e:
        exc = f"SystemExit({e.code})"
    except Exception as e:  # noqa: BLE001 - compared between the two runs
        exc = f"{type(e).__name__}{e.args}"
    return buf.getvalue(), exc, rng.getstate()


def _rank_main(rank, world, port, argv, seed, q):
    os.environ["DCR_SHARD"] = "1"
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        stats = {}
        out, exc, state = _outcome(argv, seed, stats)
        q.put((rank, out, exc, state, (stats.get("shard_rounds"), stats.get("count_pass"))))
    finally:
        dist.destroy_process_group()


def _records(path):
    with bam.AlignmentFile(path, "rb") as f:
        return [r.to_dict() for r in f]


def run_sharded(argv, seed, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, argv, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, out, exc, state, rounds = q.get(timeout=240)
        got[rank] = (out, exc, state, rounds)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def outputs(out_bam):
    base = out_bam[:-4]
    return [_records(p) for p in (out_bam, base + "_filteredreads.bam", base + "_filteredfamilies.bam")]


def compare(tmp_path, in_bam, extra, seed, world, expect_exc=None, expect_rounds=None):
    one = str(tmp_path / "one.bam")
    many = str(tmp_path / "many.bam")
    out1, exc1, st1 = _outcome(["-i", in_bam, "-o", one, *extra], seed)
    # ranks > 0 write their parts here (cli._part_dir), rank 0 the final files
    part_dir = tmp_path / "parts"
    part_dir.mkdir(exist_ok=True)
    os.environ["DCR_PART_DIR"] = str(part_dir)
    try:
        got = run_sharded(["-i", in_bam, "-o", many, *extra], seed, world)
    finally:
        del os.environ["DCR_PART_DIR"]
    out0, exc0, st0, rounds = got[0]
    assert exc1 == expect_exc
    assert exc0 == exc1
    assert out0 == out1
    assert st0 == st1
    for a, b in zip(outputs(many), outputs(one)):
        assert len(a) == len(b)
        assert a == b
    for r in range(1, world):
        assert got[r][0] == "" and got[r][1] is None        # ranks > 0 print nothing
    if expect_rounds is not None:
        assert max(g[3][0] or 0 for g in got.values()) == expect_rounds
    # nothing left behind but the three outputs
    left = sorted(p.name for p in tmp_path.iterdir() if ".part" in p.name) + sorted(p.name for p in part_dir.iterdir())
    assert left == []
    return got


@pytest.fixture(scope="module")
def filters_bam(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("shard") / "filters.bam")
    cfg = synth.SynthConfig("t", 1500, sub_size="poisson5", seed=11, low_mapq_frac=0.1, indel_frac=0.1,
                            softclip_frac=0.1)
    synth.write_config_bam(path, cfg)
    return path


def test_split_points_are_family_starts(filters_bam):
    """Ranges between split points hold exactly the single run's families."""
    p = ConsensusParams(min_reads=3)

    def fams(start, end):
        ing = native_io.Ingest(filters_bam, p.min_map_quality, p.min_reads, p.max_reads, p.min_base_quality, 0,
                               start, end)
        codes = []
        while True:
            hb = native_io.HostBatch(reads=1 << 15)
            ing.next(hb)
            for t in range(hb.s.n_tab):
                o = e = int(hb.a["tab_code"][t])
                while hb.a["names"][e]:
                    e += 1
                codes.append(bytes(hb.a["names"][o:e]))
            if hb.end_kind != native_io.END_FULL:
                break
        c = ing.counters()
        ing.close()
        return codes, c

    full, cf = fams(0, -1)
    for n in (2, 3, 4, 7):
        sp = native_io.split_points(filters_bam, n, p)
        assert all(v > 0 for v in sp)
        assert sp == sorted(sp)
        pts = [0] + sp + [-1]
        codes, tot = [], {}
        for a, b in zip(pts[:-1], pts[1:]):
            c, k = fams(a, b)
            codes += c
            for key, v in k.items():
                tot[key] = tot.get(key, 0) + v
        assert codes == full
        assert tot == cf


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_filters_and_summary(tmp_path, filters_bam, world):
    compare(tmp_path, filters_bam, ["--min_reads", "3", "-v"], 5, world, expect_rounds=1)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_downsampling_random_states(tmp_path, filters_bam, world):
    # subfamilies above --max_reads 3 are sampled in every range: ranks > 0
    # wait at their first sample call for the exact state, and none runs twice
    got = compare(tmp_path, filters_bam, ["--max_reads", "3"], 7, world, expect_rounds=1)
    # the last rank's calls are read by nobody: it never counts
    assert got[world - 1][3][1] is False


def test_sharded_no_downsampling_counts_nothing(tmp_path, filters_bam):
    # nothing above --max_reads: no rank asks for a state, no count pass runs
    got = compare(tmp_path, filters_bam, ["--max_reads", "1000"], 7, 3, expect_rounds=1)
    assert all(g[3][1] is False for g in got.values())


@pytest.mark.parametrize("where,extra", [(0.2, []), (0.8, []), (0.2, ["--max_reads", "3"]), (0.8, ["--max_reads", "3"])])
def test_sharded_reference_stop(tmp_path, filters_bam, where, extra):
    # a read without RX: pass_filters prints and exits (:1135-1181) there
    recs = list(bam.AlignmentFile(filters_bam, "rb"))
    k = int(len(recs) * where)
    while recs[k].mapping_quality < 20:
        k += 1
    recs[k]._tags = [t for t in recs[k]._tags if t[0] != "RX"]
    path = str(tmp_path / "stop.bam")
    with bam.AlignmentFile(filters_bam, "rb") as src:
        hdr = src.header
    with bam.AlignmentFile(path, "wb", header=hdr) as out:
        for r in recs:
            out.write(r)
    compare(tmp_path, path, ["--min_reads", "3", *extra], 3, 2, expect_exc="SystemExit(1)")


def test_state_exchange_failure_marker():
    """A rank that fails before it knows its random.sample calls publishes a
    failure marker: a later rank's gate raises at once instead of waiting up
    to the store timeout for calls that never come."""
    import types
    from duplexumiconsensusreads_amd import cli

    class Store:
        def __init__(self):
            self.kv = {}

        def set(self, k, v):
            self.kv[k] = v

        def get(self, k):
            return self.kv[k]

        def wait(self, keys, timeout=None):
            missing = [k for k in keys if k not in self.kv]
            if missing:
                raise TimeoutError(missing)

    store = Store()
    dist = types.SimpleNamespace(distributed_c10d=types.SimpleNamespace(_get_default_store=lambda: store))
    s0 = random.Random(3).getstate()
    r0 = cli._StateExchange(dist, 0, 2, s0, None, None, None, 1)
    r1 = cli._StateExchange(dist, 1, 2, s0, None, None, None, 1)
    r1.pre = r0.pre
    r0.publish(None)
    with pytest.raises(RuntimeError, match="failed before publishing"):
        r1.gate()
    r0.published = False
    r0.publish([(10, 3)])
    want = random.Random()
    want.setstate(s0)
    want.sample(range(10), 3)
    assert r1.gate() == want.getstate()


@pytest.mark.parametrize("mapped", [True, False])
def test_write_part_at_places_the_part_byte_for_byte(tmp_path, mapped):
    """The merge's part copy (cli._write_part_at): into a preallocated range
    through a mapping (unaligned offsets, parts larger than one slice) or by
    pwrite, the final file holds its prefix and then the part's first n bytes."""
    rng = random.Random(7)
    for n, off in [(1, 0), (5000, 12345), (3 << 20, 4097), (9 << 20, 65535)]:
        data = rng.randbytes(n)
        part, final = tmp_path / "p.part", tmp_path / "f.bam"
        part.write_bytes(data + b"tail")
        head = rng.randbytes(off)
        final.write_bytes(head)
        if mapped:
            fd = os.open(final, os.O_RDWR)
            try:
                os.posix_fallocate(fd, off, n)
            finally:
                os.close(fd)
        cli._write_part_at(str(part), str(final), n, off, mapped=mapped)
        assert final.read_bytes() == head + data
