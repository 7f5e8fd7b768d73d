"""The native host side (libdcr_io.so, include/dcr_io.h) on CPU:

* the library exports every function the header declares and the ctypes
  mirror of ``dcr_host_batch`` has the header's layout;
* CPython's ``random.sample`` restated natively (MT19937 state in / out),
  both of its branches (pool and set), against the interpreter;
* the ingest (filters, MI grouping, family checks, split, downsampling,
  packing, side records) against the host's Python restatement of the same
  steps (cli.pass_filters / pipeline.prepare_family / batch.pack_families),
  array for array and byte for byte, across batch sizes;
* truncated and malformed input fail loudly.
"""
import ctypes
import os
import random
import re
import subprocess

import numpy as np
import pytest

from duplexumiconsensusreads_amd import bam, native_io, synth

from .harness import pipeline
from duplexumiconsensusreads_amd.batch import BATCH_FIELDS, pack_families
from duplexumiconsensusreads_amd.params import ConsensusParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dcr_io.h")
GOLDEN_BAM = os.path.join(ROOT, "tests", "golden", "e2e_c1_small.bam")


def test_library_exports_every_header_function():
    lib = native_io.load()
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    names = sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(dcr_\w+)\s*\(", txt, flags=re.M)))
    assert "dcr_ingest_next" in names and "dcr_fmt_write" in names
    for n in names:
        assert hasattr(lib, n), n


def test_host_batch_layout_matches_header():
    src = (f'#include "{HEADER}"\n#include <stdio.h>\n#include <stddef.h>\n'
           'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(dcr_host_batch), offsetof(dcr_host_batch, n_fam),'
           ' offsetof(dcr_host_batch, err_msg), sizeof(dcr_ingest_cfg));return 0;}\n')
    exe = "/tmp/_dcr_io_sizeof"
    subprocess.run(["gcc", "-x", "c", "-", "-o", exe], input=src, text=True, check=True)
    got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    S = native_io.HostBatchStruct
    assert got == [ctypes.sizeof(S), S.n_fam.offset, S.err_msg.offset, ctypes.sizeof(native_io.IngestCfg)]


@pytest.mark.parametrize("n,k", [(5, 3), (30, 10), (150, 100), (1000, 100), (26, 6), (27, 6), (1000, 999),
                                 (50, 1), (400, 60), (2, 1)])
def test_native_sample_is_cpython_sample(n, k):
    r = random.Random(n * 1000 + k)
    for _ in range(5):
        st = r.getstate()
        got, st2 = native_io.py_sample(st, n, k)
        assert got == r.sample(range(n), k)
        assert st2 == r.getstate()


def python_ingest(path, P, seed):
    """The same steps through the Python host restatement (per record)."""
    rng = random.Random(seed)
    proc, exc, filt = [], [], []
    fam, code = None, None

    def done(f):
        res = pipeline.prepare_family(f, P, rng)
        if res.subs is None:
            filt.extend(f)
        else:
            proc.append(res.subs)

    with bam.AlignmentFile(path, "rb") as inb:
        for r in inb:
            if not legacy_pass_filters(r, P.min_map_quality):
                exc.append(r)
                continue
            c = r.get_tag("MI").split("/")[0]
            if fam is None:
                fam, code = [r], c
            elif c == code:
                fam.append(r)
            else:
                done(fam)
                fam, code = [r], c
    done(fam)
    return pack_families(proc), exc, filt, rng


def legacy_pass_filters(read, q):
    """pass_filters (:1135-1181) on a decoded record (no format errors in these inputs)."""
    return (read.is_paired and read.is_proper_pair and not read.is_unmapped and not read.mate_is_unmapped
            and not read.is_supplementary and not read.is_qcfail and read.mapping_quality >= q)


def native_ingest(path, P, seed, reads):
    rng = random.Random(seed)
    ing = native_io.Ingest(path, P.min_map_quality, P.min_reads, P.max_reads, P.min_base_quality, 4)
    ing.set_rng_state(rng.getstate())
    out = []
    while True:
        hb = native_io.HostBatch(reads=reads, side_bytes=1 << 22)
        ing.next(hb)
        pk = hb.packed()
        out.append((hb.s.n_reads, hb.s.n_bases, hb.s.n_cigar, hb.s.ss_cols, hb.s.ds_cols,
                    {k: getattr(pk, k).copy() for k in BATCH_FIELDS}, hb.side("exc").tobytes(),
                    hb.side("filt").tobytes()))
        if hb.end_kind != native_io.END_FULL:
            assert hb.end_kind == native_io.END_EOF
            break
    rng.setstate(ing.rng_state(rng.getstate()))
    counters = ing.counters()
    ing.close()
    return out, rng, counters


def concat(out):
    cat = {k: [] for k in BATCH_FIELDS}
    ro = bo = co = so = do = 0
    for n_reads, n_bases, n_cig, ss_cols, ds_cols, a, _, _ in out:
        for k, base in (("sub_off", ro), ("ss_col_off", so), ("ds_col_off", do)):
            cat[k].append(a[k][1:] + base if cat[k] else a[k] + base)
        for k in ("read_pos", "read_mapq", "seq_len", "cig_n", "cigar", "bases", "quals"):
            cat[k].append(a[k])
        cat["seq_off"].append(a["seq_off"] + bo)
        cat["cig_off"].append(a["cig_off"] + co)
        ro, bo, co, so, do = ro + n_reads, bo + n_bases, co + n_cig, so + ss_cols, do + ds_cols
    return {k: np.concatenate(v) for k, v in cat.items()}


@pytest.fixture(scope="module")
def c1_bam(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("ing") / "c1.bam")
    cfg = synth.SynthConfig("t", 600, sub_size="poisson5", indel_frac=0.1, softclip_frac=0.1, seed=5)
    synth.write_config_bam(path, cfg)
    return path


@pytest.mark.parametrize("which,seed,max_reads,min_reads,reads", [
    ("golden", 1, 100, 1, 1 << 16), ("golden", 7, 3, 1, 300), ("golden", 3, 6, 4, 200),
    ("c1", 11, 7, 3, 5000), ("c1", 12, 4, 2, 1 << 20)])
def test_ingest_matches_python_host_path(c1_bam, which, seed, max_reads, min_reads, reads):
    path = GOLDEN_BAM if which == "golden" else c1_bam
    P = ConsensusParams(max_reads=max_reads, min_reads=min_reads)
    pk, exc, filt, rng1 = python_ingest(path, P, seed)
    out, rng2, counters = native_ingest(path, P, seed, reads)
    assert rng1.getstate() == rng2.getstate()
    got = concat(out)
    for k in BATCH_FIELDS:
        assert np.array_equal(got[k], getattr(pk, k)), k
    assert b"".join(o[6] for o in out) == b"".join(bam.encode_record(r) for r in exc)
    assert b"".join(o[7] for o in out) == b"".join(bam.encode_record(r) for r in filt)
    assert counters["excluded"] == len(exc) and counters["processed"] == pk.n_fam


def test_ingest_rejects_truncated_input(tmp_path):
    data = bam.bgzf_stream(GOLDEN_BAM)
    bad = str(tmp_path / "trunc.bam")
    w = bam.BGZFWriter(bad)
    w.write(data[:len(data) - 100])          # ends inside a record
    w.close()
    ing = native_io.Ingest(bad)
    hb = native_io.HostBatch(reads=1 << 16, side_bytes=1 << 22)
    with pytest.raises(native_io.IOError_, match="truncated"):
        ing.next(hb)
    with pytest.raises(ValueError, match="truncated"):
        with bam.AlignmentFile(bad, "rb") as f:
            list(f)


def test_ingest_rejects_non_bam(tmp_path):
    p = tmp_path / "x.bam"
    p.write_bytes(b"not a bam at all" * 10)
    with pytest.raises(native_io.IOError_):
        native_io.Ingest(str(p))


def test_bgzf_writer_rewrites_a_longer_file(tmp_path):
    """A rewrite over a longer file of the same name gives the bytes of a
    fresh one; a writer dropped before close leaves no stale tail (the file
    is truncated at open, so no old BGZF EOF marker survives)."""
    import gzip
    small, big = b"BAM\x01" + bytes(range(256)) * 4, os.urandom(3 << 20)
    fresh, reused = tmp_path / "fresh.bam", tmp_path / "reused.bam"
    w = native_io.BgzfWriter(str(reused), big, 1, 2)
    w.close()
    assert reused.stat().st_size > 3 << 20
    for path in (fresh, reused):
        w = native_io.BgzfWriter(str(path), small, 1, 2)
        w.close()
    assert reused.read_bytes() == fresh.read_bytes()
    assert gzip.decompress(reused.read_bytes()) == small
    # dropped before close over the longer file: nothing of the old file left
    w = native_io.BgzfWriter(str(reused), big, 1, 2)
    w.close()
    w = native_io.BgzfWriter(str(reused), small, 1, 2)
    assert reused.stat().st_size < 1 << 20
    assert not reused.read_bytes().endswith(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    w.close()


def test_bgzf_writer_non_regular_outputs(tmp_path):
    """Outputs that are not regular files: a symlink to /dev/null and a FIFO."""
    import gzip
    import threading
    data = b"BAM\x01" + os.urandom(1 << 18)
    link = tmp_path / "null.bam"
    os.symlink("/dev/null", link)
    w = native_io.BgzfWriter(str(link), data, 6, 2)
    w.close()
    fifo = tmp_path / "pipe.bam"
    os.mkfifo(fifo)
    got = []
    th = threading.Thread(target=lambda: got.append(open(fifo, "rb").read()))
    th.start()
    w = native_io.BgzfWriter(str(fifo), data, 6, 2)
    w.close()
    th.join(30)
    assert gzip.decompress(got[0]) == data


def _ingest_all(path, P, setup):
    ing = native_io.Ingest(path, P.min_map_quality, P.min_reads, P.max_reads, P.min_base_quality, 2)
    setup(ing)
    bases = []
    while True:
        hb = native_io.HostBatch(reads=1 << 14, side_bytes=1 << 22)
        ing.next(hb)
        bases.append(hb.packed().bases.copy())
        if hb.end_kind != native_io.END_FULL:
            break
    calls = ing.sample_calls()
    ing.close()
    return np.concatenate(bases), calls


def test_state_gate(c1_bam):
    """dcr_ingest_set_state_gate: called once, right before the first
    random.sample call, and sampling then runs from the state it returns --
    the same reads as an ingest started from that state."""
    P = ConsensusParams(max_reads=3)
    want_state = random.Random(99).getstate()
    want, calls_w = _ingest_all(c1_bam, P, lambda ing: ing.set_rng_state(want_state))
    seen = []

    def setup(ing):
        ing.set_rng_state(random.Random(1).getstate())     # a state the gate replaces
        ing.set_state_gate(lambda: (seen.append(len(ing.sample_calls())), want_state)[1])
    got, calls_g = _ingest_all(c1_bam, P, setup)
    assert calls_w and calls_g == calls_w
    assert seen == [0]                                     # once, before the first call
    assert np.array_equal(got, want)
    # an ingest that never samples never calls its gate
    seen.clear()
    _ingest_all(c1_bam, ConsensusParams(max_reads=1000), setup)
    assert seen == []


def test_state_gate_error_ends_ingest(c1_bam):
    P = ConsensusParams(max_reads=3)
    ing = native_io.Ingest(c1_bam, P.min_map_quality, P.min_reads, P.max_reads, P.min_base_quality, 2)

    def bad():
        raise RuntimeError("no state")
    ing.set_state_gate(bad)
    with pytest.raises(native_io.IOError_):
        while True:
            hb = native_io.HostBatch(reads=1 << 14, side_bytes=1 << 22)
            ing.next(hb)
            if hb.end_kind != native_io.END_FULL:
                break
    assert isinstance(ing.gate_error, RuntimeError)
    ing.close()


def test_ingest_many_chunks_reproduces_the_source_batch(tmp_path):
    """A BAM of ~3.2 M reads (a dozen 32 MiB inflate chunks, so families
    straddle chunk windows and the serial-scan buffer) read back through the
    native ingest in 512 k-read batches: the packed reads of every batch,
    concatenated, are exactly the batch the BAM was written from.  Families
    are completed on the packer thread while the walk moves on, and the
    chunk windows their records point into are retired only after them."""
    src = synth.packed_fixed_size(100_000, seed=9)
    path = str(tmp_path / "many.bam")
    synth.write_packed_bam(path, src, seed=9, level=1)
    ing = native_io.Ingest(path, 20, 1, 100, 20, 4)
    got = {k: [] for k in ("read_pos", "seq_len", "cig_n", "bases", "quals")}
    n_fam = 0
    while True:
        hb = native_io.HostBatch(reads=1 << 19)
        ing.next(hb)
        pk = hb.packed()
        n_fam += pk.n_fam
        for k in got:
            got[k].append(getattr(pk, k).copy())
        if hb.end_kind != native_io.END_FULL:
            assert hb.end_kind == native_io.END_EOF
            break
    ing.close()
    assert n_fam == src.n_fam
    for k, v in got.items():
        assert np.array_equal(np.concatenate(v), getattr(src, k)), k


def test_ingest_long_mismatched_rx_stays_in_the_names_buffer(tmp_path):
    """A family whose first A1 / B1 reads carry RX strings much longer than
    its first record's (the UMI check fails, but only on the packer task,
    after the walk has reserved the family's names): the reservation counts
    the RX that is actually written, so a batch near its names capacity ends
    before the family instead of writing past the buffer, and the family
    then fails the UMI check in the next batch as the reference does (:110)."""
    from duplexumiconsensusreads_amd.bam import AlignmentFile, BamHeader
    from duplexumiconsensusreads_amd.records import AlignedSegment

    def rec(name, flag, mi, rx, pos=100):
        r = AlignedSegment()
        r.query_name, r.flag, r.reference_id, r.reference_start = name, flag, 0, pos
        r.mapping_quality = 60
        r.cigartuples = [(0, 20)]
        r.query_sequence = "ACGT" * 5
        r.query_qualities = [30] * 20
        r.next_reference_id, r.next_reference_start = 0, pos
        r.set_tags([("MI", mi), ("RX", rx)])
        return r

    fams = []
    for k in range(15):                      # 60 reads, ~6 KB of names
        rx = "A" * 100 + "-" + "C" * 99
        fams.append([rec(f"q{k}_{j}", fl, f"{k}/{'A' if fl in (99, 147) else 'B'}", rx)
                     for j, fl in enumerate((99, 163, 83, 147))])
    big = "G" * 16450 + "-" + "T" * 16449    # 32,900 bytes per RX
    fams.append([rec("x0", 147, "15/A", "AC-GT"), rec("x1", 99, "15/A", big), rec("x2", 83, "15/B", big),
                 rec("x3", 163, "15/B", "AC-GT")])
    path = str(tmp_path / "longrx.bam")
    hdr = BamHeader("@HD\tVN:1.6\n@SQ\tSN:chr1\tLN:1000000\n", ["chr1"], [1000000])
    with AlignmentFile(path, "wb", header=hdr) as out:
        for fam in fams:
            for r in fam:
                out.write(r)
    guard = 1 << 20

    def guarded(nbytes):
        buf = np.full(nbytes + guard, 0xA5, np.uint8)
        guarded.bufs.append((buf, nbytes))
        return buf[:nbytes]
    guarded.bufs = []
    ing = native_io.Ingest(path, 20, 1, 100, 20, 2)
    kinds = []
    while True:
        hb = native_io.HostBatch(reads=64, side_bytes=1 << 20, alloc=guarded)
        ing.next(hb)
        kinds.append((hb.s.n_fam, hb.end_kind))
        if hb.end_kind != native_io.END_FULL:
            break
    err = hb.error()
    ing.close()
    for buf, n in guarded.bufs:
        assert (buf[n:] == 0xA5).all(), "write past the batch's arrays"
    assert kinds[0] == (15, native_io.END_FULL)
    assert kinds[-1][1] != native_io.END_EOF and "UMI" in err[1].upper(), (kinds, err)
