"""Synthetic duplex-UMI inputs for the five BASELINE.json configs.

Two generators with the same distribution:

* ``family_records`` builds pysam-style records (for BAM files, the end-to-end
  CLI path and the reference-run golden vectors);
* ``packed_config`` builds a device batch directly in the packed columnar
  layout (for the bench at 10 M+ reads, where per-record Python is too slow).

Family layout follows the fgbio GroupReadsByUmi output the reference expects
(DuplexUMIConsensusReads.py:132-154, :1185-1217): reads of one MI family are
contiguous; A1/B2 map forward at P, B1/A2 reverse at P+I-L; MI is ``k/A`` on
A1/A2 and ``k/B`` on B1/B2; RX is ``U1-U2`` on A and ``U2-U1`` on B.
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np

from .records import AlignedSegment

_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
# flags: paired|proper + strand/mate + read1/read2
FLAG_A1, FLAG_B2, FLAG_B1, FLAG_A2 = 99, 163, 83, 147


@dataclasses.dataclass
class SynthConfig:
    name: str
    n_families: int
    read_len: int = 150
    sub_size: str = "poisson5"       # poisson5 | fixed8 | zipf | loguniform | poisson4p1
    fixed_size: int = 8
    zipf_s: float = 1.5
    zipf_max: int = 100
    logu_lo: int = 100
    logu_hi: int = 1000
    indel_frac: float = 0.0          # reads carrying one I or D of 1-3 bp at offset 20-130
    softclip_frac: float = 0.0       # reads carrying a 1-10 bp soft clip
    low_mapq_frac: float = 0.02
    seed: int = 1
    n_loci: int = 0                  # >0: families share these loci (deep panel)


CONFIGS = {
    "C1": SynthConfig("C1", 1000, sub_size="poisson5", seed=1),
    "C2": SynthConfig("C2", 312_500, sub_size="fixed8", fixed_size=8, low_mapq_frac=0.0, seed=2),
    "C3": SynthConfig("C3", 0, sub_size="zipf", indel_frac=0.05, softclip_frac=0.03, seed=3),
    "C4": SynthConfig("C4", 1000, sub_size="loguniform", n_loci=20, seed=4),
    "C5": SynthConfig("C5", 0, sub_size="poisson4p1", seed=5),
}


def _sub_sizes(rng, cfg, n):
    if cfg.sub_size == "fixed8":
        return np.full(n, cfg.fixed_size, dtype=np.int64)
    if cfg.sub_size == "poisson5":
        return np.clip(rng.poisson(5, n), 1, 12)
    if cfg.sub_size == "poisson4p1":
        return rng.poisson(4, n) + 1
    if cfg.sub_size == "zipf":
        k = np.arange(1, cfg.zipf_max + 1)
        p = k ** -cfg.zipf_s
        p /= p.sum()
        return rng.choice(k, size=n, p=p)
    if cfg.sub_size == "loguniform":
        return np.exp(rng.uniform(np.log(cfg.logu_lo), np.log(cfg.logu_hi), n)).astype(np.int64)
    raise ValueError(cfg.sub_size)


def _quals(rng, n):
    u = rng.random(n)
    q = np.where(u < 0.80, 37, np.where(u < 0.92, 25, 12)).astype(np.uint8)
    return q


def _mutate(rng, tmpl, q):
    """Substitute bases at the phred error rate 10^(-Q/10)."""
    err = rng.random(len(tmpl)) < 10.0 ** (-q.astype(np.float64) / 10.0)
    out = tmpl.copy()
    if err.any():
        shift = rng.integers(1, 4, err.sum())
        idx = np.searchsorted(_ACGT, out[err])
        out[err] = _ACGT[(idx + shift) % 4]
    return out


def _one_read(rng, cfg, tmpl_fwd, start, L, reverse):
    """Bases/quals/cigar of one read copied from the family template."""
    q = _quals(rng, L)
    if not (q >= 20).any():
        q[rng.integers(0, L)] = 37
    cigar = [(0, L)]
    shift = 0
    seq = tmpl_fwd[start:start + L].copy()
    if cfg.indel_frac and rng.random() < cfg.indel_frac:
        off = int(rng.integers(20, min(131, L - 5)))
        ln = int(rng.integers(1, 4))
        if rng.random() < 0.5:   # insertion: ln extra bases inside the read
            ins = _ACGT[rng.integers(0, 4, ln)]
            seq = np.concatenate([seq[:off], ins, seq[off:L - ln]])
            cigar = [(0, off), (1, ln), (0, L - off - ln)]
        else:                    # deletion: skip ln template bases
            seq = np.concatenate([seq[:off], tmpl_fwd[start + off + ln:start + L + ln]])
            cigar = [(0, off), (2, ln), (0, L - off)]
    if cfg.softclip_frac and rng.random() < cfg.softclip_frac:
        sc = int(rng.integers(1, 11))
        if rng.random() < 0.5:
            ops = [(4, sc)] + cigar
            ops[1] = (0, ops[1][1] - sc)
            shift = sc
        else:
            ops = cigar[:-1] + [(0, cigar[-1][1] - sc), (4, sc)]
        cigar = ops
    seq = _mutate(rng, seq, q)
    return seq, q, cigar, shift


def family_records(rng, cfg: SynthConfig, fam_id: int, tid=0, locus=None):
    """Records of one duplex family in BAM order (pairs adjacent)."""
    L = cfg.read_len
    n4 = _sub_sizes(rng, cfg, 4)
    ins = max(int(np.clip(rng.normal(300, 30), 200, 500)), L + 10)
    P = int(locus if locus is not None else rng.integers(1000, 100_000_000))
    tmpl = _ACGT[rng.integers(0, 4, ins + 20)]
    u1 = "".join(chr(c) for c in _ACGT[rng.integers(0, 4, 8)])
    u2 = "".join(chr(c) for c in _ACGT[rng.integers(0, 4, 8)])
    recs = []
    # subfamily -> (flag, strand tag, reverse?, rx)
    spec = [(FLAG_A1, "A", False), (FLAG_B2, "B", False), (FLAG_B1, "B", True), (FLAG_A2, "A", True)]
    for k, (flag, strand, rev) in enumerate(spec):
        for j in range(int(n4[k])):
            start = 0 if not rev else ins - L
            seq, q, cig, shift = _one_read(rng, cfg, tmpl, start, L, rev)
            r = AlignedSegment()
            r.query_name = f"mol{fam_id}_{k}_{j}"
            r.flag = flag
            r.reference_id = tid
            r.reference_start = P + start + shift
            mq = int(rng.integers(20, 61))
            if rng.random() < cfg.low_mapq_frac:
                mq = int(rng.integers(0, 20))
            r.mapping_quality = mq
            r.cigartuples = cig
            r.query_sequence = seq.tobytes().decode()
            r.query_qualities = q.tolist()
            r.next_reference_id = tid
            r.next_reference_start = P + (ins - L if not rev else 0)
            r.template_length = ins if not rev else -ins
            rx = f"{u1}-{u2}" if strand == "A" else f"{u2}-{u1}"
            r.set_tags([("MI", f"{fam_id}/{strand}"), ("RX", rx)])
            recs.append(r)
    return recs


def write_config_bam(path, cfg: SynthConfig, n_families=None, seed=None):
    """Write a synthetic duplex BAM (families contiguous, coordinate-agnostic)."""
    from .bam import AlignmentFile, BamHeader
    rng = np.random.default_rng(cfg.seed if seed is None else seed)
    hdr = BamHeader("@HD\tVN:1.6\tSO:unsorted\n@SQ\tSN:chr1\tLN:248956422\n", ["chr1"], [248956422])
    n = cfg.n_families if n_families is None else n_families
    with AlignmentFile(path, "wb", header=hdr) as out:
        for f in range(n):
            locus = None
            if cfg.n_loci:
                locus = 1_000_000 + 10_000 * (f % cfg.n_loci)
            for r in family_records(rng, cfg, f, locus=locus):
                out.write(r)
    return path


def write_packed_bam(path, packed, seed=0, level=1, n_threads=0, chunk_families=1 << 16, header=True, fam_id0=0):
    """Write the families of a packed batch (``packed_fixed_size`` /
    ``packed_config``) as a duplex BAM through the native record writer
    (include/dcr_io.h dcr_synth_write): the bench's 10 M+-read inputs.  UMIs
    are random per family (seeded); every read passes the reference's filters
    (paired, proper, MAPQ >= 20 as generated).  header=False: the records'
    BGZF blocks only (plus the EOF block), a piece of a larger BAM; fam_id0:
    the MI code of its first family (pieces of one BAM keep codes distinct)."""
    from . import native_io
    from .batch import PackedBatch
    hdr = BamHeader_bytes() if header else b""
    w = native_io.BgzfWriter(path, hdr, level=level, n_threads=n_threads)
    rng = np.random.default_rng(seed)
    F = packed.n_fam
    for f0 in range(0, F, chunk_families):
        f1 = min(F, f0 + chunk_families)
        r0, r1 = int(packed.sub_off[4 * f0]), int(packed.sub_off[4 * f1])
        c0 = int(packed.cig_off[r0]) if r1 > r0 else 0
        part = PackedBatch.__new__(PackedBatch)
        part.sub_off = (packed.sub_off[4 * f0:4 * f1 + 1] - r0).astype(np.int32)
        part.read_pos, part.read_mapq = packed.read_pos[r0:r1], packed.read_mapq[r0:r1]
        part.seq_off, part.seq_len = packed.seq_off[r0:r1], packed.seq_len[r0:r1]
        part.cig_off, part.cig_n = (packed.cig_off[r0:r1] - c0).astype(np.int32), packed.cig_n[r0:r1]
        part.cigar = packed.cigar[c0:]
        part.bases, part.quals = packed.bases, packed.quals
        part.n_fam, part.n_reads = f1 - f0, r1 - r0
        umis = _ACGT[rng.integers(0, 4, 16 * (f1 - f0))]
        w.write_synthetic(part, umis, fam_id0=fam_id0 + f0, n_threads=n_threads)
    w.close()
    return path


def BamHeader_bytes():
    from .bam import BamHeader
    return BamHeader("@HD\tVN:1.6\tSO:unsorted\n@SQ\tSN:chr1\tLN:248956422\n", ["chr1"], [248956422]).encode()


def split_records(recs):
    """Four subfamilies in A1, B2, B1, A2 order (split_family :132-154)."""
    out = [[], [], [], []]
    for r in recs:
        if not r.is_reverse and r.is_read1:
            out[0].append(r)
        elif not r.is_reverse and r.is_read2:
            out[1].append(r)
        elif r.is_reverse and r.is_read1:
            out[2].append(r)
        elif r.is_reverse and r.is_read2:
            out[3].append(r)
    return out


def family_splits(cfg: SynthConfig, n_families=None, seed=None):
    rng = np.random.default_rng(cfg.seed if seed is None else seed)
    n = cfg.n_families if n_families is None else n_families
    fams = []
    for f in range(n):
        locus = 1_000_000 + 10_000 * (f % cfg.n_loci) if cfg.n_loci else None
        fams.append(split_records(family_records(rng, cfg, f, locus=locus)))
    return fams


def packed_from_records(cfg: SynthConfig, n_families=None, seed=None):
    """Packed batch through the record generator (any config, moderate sizes)."""
    from .batch import pack_families
    return pack_families(family_splits(cfg, n_families, seed))


_QLUT = np.array([37] * 80 + [25] * 12 + [12] * 8, dtype=np.uint8)
_ERR_P16 = {37: int(round(10 ** -3.7 * 65536)), 25: int(round(10 ** -2.5 * 65536)),
            12: int(round(10 ** -1.2 * 65536))}


def packed_fixed_size(n_families, sub_size=8, read_len=150, seed=2, chunk_reads=1 << 18, threads=None):
    """Vectorised config-2 generator: uniform subfamily size, ``150M`` reads,
    no indels.  Same base/quality model as family_records.
    Chunks of families are filled by a thread pool (numpy releases the GIL),
    each from its own generator seeded by (seed, chunk): the bytes depend on
    ``seed`` and ``chunk_reads`` only, not on the thread count."""
    from concurrent.futures import ThreadPoolExecutor

    from .batch import finish_batch
    rng = np.random.default_rng(seed)
    F, L, k = n_families, read_len, sub_size
    n = F * 4 * k
    ins = np.clip(rng.normal(300, 30, F), 200, 500).astype(np.int64)
    P = rng.integers(1000, 100_000_000, F).astype(np.int64)
    sub = np.repeat(np.arange(4), k)
    rev = sub >= 2
    start = np.where(rev[None, :], ins[:, None] - L, 0).reshape(-1)       # [n]
    read_pos = (np.repeat(P, 4 * k) + start).astype(np.int32)
    tw = int(ins.max()) + 20 if F else L
    bases = np.empty(n * L, np.uint8)
    quals = np.empty(n * L, np.uint8)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    err_lut = np.zeros(256, np.uint16)
    for q, v in _ERR_P16.items():
        err_lut[q] = v
    fam_chunk = max(1, chunk_reads // (4 * k))
    ar = np.arange(L)

    def fill(ci):
        f0 = ci * fam_chunk
        f1 = min(F, f0 + fam_chunk)
        g = np.random.default_rng([seed, ci])
        tmpl = acgt[g.integers(0, 4, (f1 - f0) * tw, dtype=np.uint8)]
        r0, r1 = f0 * 4 * k, f1 * 4 * k
        idx = (np.repeat(np.arange(f1 - f0) * tw, 4 * k) + start[r0:r1])[:, None] + ar[None, :]
        seq = tmpl[idx]
        q = _QLUT[g.integers(0, 100, (r1 - r0, L), dtype=np.uint8)]
        err = g.integers(0, 65536, (r1 - r0, L), dtype=np.uint16) < err_lut[q]
        if err.any():
            code = np.searchsorted(acgt, seq[err])
            seq[err] = acgt[(code + g.integers(1, 4, int(err.sum()))) % 4]
        bases[r0 * L:r1 * L] = seq.reshape(-1)
        quals[r0 * L:r1 * L] = q.reshape(-1)

    n_chunks = (F + fam_chunk - 1) // fam_chunk
    with ThreadPoolExecutor(threads or min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(fill, range(n_chunks)))
    sub_off = np.arange(0, n + 1, k, dtype=np.int32)
    mapq = rng.integers(20, 61, n).astype(np.uint8)
    seq_off = np.arange(n, dtype=np.int64) * L
    seq_len = np.full(n, L, np.int32)
    cig_off = np.arange(n, dtype=np.int32)
    cig_n = np.ones(n, np.int32)
    cigar = np.full(n, (L << 4) | 0, np.uint32)
    return finish_batch(sub_off, read_pos, mapq, seq_off, seq_len, cig_off, cig_n, cigar, bases, quals)


def config_family_reads(cfg: SynthConfig, n_families=None, seed=None, max_reads=None):
    """Reads per family of ``packed_config``'s stream (its first draw), for
    planning a split of the stream before generating it."""
    rng = np.random.default_rng(cfg.seed if seed is None else seed)
    F = cfg.n_families if n_families is None else n_families
    sizes = _sub_sizes(rng, cfg, 4 * F).astype(np.int64)
    if max_reads is not None:
        sizes = np.minimum(sizes, max_reads)
    return sizes.reshape(F, 4).sum(1)


def packed_config(cfg: SynthConfig, n_families=None, seed=None, max_reads=None, chunk_reads=1 << 18,
                  threads=None, keep=None):
    """Vectorised generator for any config shape: subfamily
    sizes from ``cfg.sub_size`` (capped at ``max_reads``, the downsampling the
    host would have applied), one I or D of 1-3 bp at offset 20-130 on
    ``indel_frac`` of the reads, a 1-10 bp soft clip at either end on
    ``softclip_frac`` of them, deep-panel loci when ``cfg.n_loci``.  Same base
    / quality / substitution model as ``family_records``; reads are the ones
    that passed ``pass_filters`` (MAPQ 20..60).  For bench-scale batches of
    the C3 / C4 / C5 shapes, where the per-record generator is too slow.
    ``keep`` (increasing family indices) returns only those families, the
    same bytes as in the whole stream (a rank's share of a shared stream)."""
    from concurrent.futures import ThreadPoolExecutor

    from .batch import finish_batch, subset_families
    rng = np.random.default_rng(cfg.seed if seed is None else seed)
    F = cfg.n_families if n_families is None else n_families
    L = cfg.read_len
    sizes = _sub_sizes(rng, cfg, 4 * F).astype(np.int64)
    if max_reads is not None:
        sizes = np.minimum(sizes, max_reads)
    sub_off = np.zeros(4 * F + 1, np.int64)
    sub_off[1:] = np.cumsum(sizes)
    n = int(sub_off[-1])
    sub_of = np.repeat(np.arange(4 * F), sizes)
    fam = sub_of // 4
    rev = (sub_of % 4) >= 2
    ins = np.maximum(np.clip(rng.normal(300, 30, F), 200, 500).astype(np.int64), L + 10)
    if cfg.n_loci:
        P = 1_000_000 + 10_000 * (np.arange(F) % cfg.n_loci)
    else:
        P = rng.integers(1000, 100_000_000, F)
    start = np.where(rev, ins[fam] - L, 0)
    # indels: kind 0 none, 1 insertion, 2 deletion
    kind = np.where(rng.random(n) < cfg.indel_frac, np.where(rng.random(n) < 0.5, 1, 2), 0)
    ioff = rng.integers(20, min(131, L - 5), n)
    iln = rng.integers(1, 4, n)
    clip = np.where(rng.random(n) < cfg.softclip_frac, rng.integers(1, 11, n), 0)
    cleft = rng.random(n) < 0.5
    # CIGAR ops per read: [S] M [I|D M] [S]
    ops = np.full((n, 5), -1, np.int64)
    lens = np.zeros((n, 5), np.int64)
    m1 = np.where(kind == 0, L, ioff)
    m2 = np.where(kind == 1, L - ioff - iln, L - ioff)
    ops[:, 1], lens[:, 1] = 0, m1
    has2 = kind > 0
    ops[has2, 2], lens[has2, 2] = kind[has2], iln[has2]
    ops[has2, 3], lens[has2, 3] = 0, m2[has2]
    lc = (clip > 0) & cleft
    rc = (clip > 0) & ~cleft
    ops[lc, 0], lens[lc, 0] = 4, clip[lc]
    lens[lc, 1] -= clip[lc]
    ops[rc, 4], lens[rc, 4] = 4, clip[rc]
    last = np.where(has2, 3, 1)
    lens[rc, last[rc]] -= clip[rc]
    live = ops >= 0
    cig_n = live.sum(1).astype(np.int32)
    cigar = ((lens[live] << 4) | ops[live]).astype(np.uint32)
    cig_off = np.zeros(n, np.int32)
    cig_off[1:] = np.cumsum(cig_n[:-1])
    read_pos = (P[fam] + start + np.where(lc, clip, 0)).astype(np.int32)
    mapq = rng.integers(20, 61, n).astype(np.uint8)
    seq_len = np.full(n, L, np.int32)
    seq_off = np.arange(n, dtype=np.int64) * L
    bases = np.empty(n * L, np.uint8)
    quals = np.empty(n * L, np.uint8)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    err_lut = np.zeros(256, np.uint16)
    for q, v in _ERR_P16.items():
        err_lut[q] = v
    tw = int(ins.max()) + 20 if F else L
    ar = np.arange(L)
    # chunks of whole families, each from its own generator
    fam_first_read = sub_off[0::4]
    fam_chunk = max(1, chunk_reads // max(1, int(np.mean(sizes)) * 4))
    n_chunks = (F + fam_chunk - 1) // fam_chunk

    def fill(ci):
        f0, f1 = ci * fam_chunk, min(F, (ci + 1) * fam_chunk)
        r0, r1 = int(fam_first_read[f0]), int(fam_first_read[f1])
        if r1 == r0:
            return
        g = np.random.default_rng([cfg.seed if seed is None else seed, ci])
        tmpl = acgt[g.integers(0, 4, (f1 - f0) * tw, dtype=np.uint8)]
        k, o, ln = kind[r0:r1, None], ioff[r0:r1, None], iln[r0:r1, None]
        delta = np.where((k == 1) & (ar >= o + ln), -ln, 0) + np.where((k == 2) & (ar >= o), ln, 0)
        idx = ((fam[r0:r1] - f0) * tw + start[r0:r1])[:, None] + ar[None, :] + delta
        seq = tmpl[idx]
        inserted = (k == 1) & (ar >= o) & (ar < o + ln)
        if inserted.any():
            seq[inserted] = acgt[g.integers(0, 4, int(inserted.sum()))]
        q = _QLUT[g.integers(0, 100, (r1 - r0, L), dtype=np.uint8)]
        err = g.integers(0, 65536, (r1 - r0, L), dtype=np.uint16) < err_lut[q]
        if err.any():
            code = np.searchsorted(acgt, seq[err])
            seq[err] = acgt[(code + g.integers(1, 4, int(err.sum()))) % 4]
        bases[r0 * L:r1 * L] = seq.reshape(-1)
        quals[r0 * L:r1 * L] = q.reshape(-1)

    todo = range(n_chunks) if keep is None else sorted(set(int(f) // fam_chunk for f in keep))
    with ThreadPoolExecutor(threads or min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(fill, todo))
    packed = finish_batch(sub_off.astype(np.int32), read_pos, mapq, seq_off, seq_len, cig_off, cig_n, cigar, bases,
                          quals)
    return packed if keep is None else subset_families(packed, keep)
