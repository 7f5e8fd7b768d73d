"""Packed columnar batch layout shared by the host, the HIP library and the
C oracle (``dcr_batch`` / ``dcr_out`` in include/dcr.h).

A batch holds F families; subfamily s = 4f + k, k = A1, B2, B1, A2 — the
order of split_family (DuplexUMIConsensusReads.py:132-154) and of the four
single-strand calls (:1564-1569).  Duplex pairs are p = 2f + j with
j = 0: (A1, B2) and j = 1: (B1, A2) (:1575-1576).

Output regions: every consensus gets a region of ``T_ub`` columns (rounded
up to a multiple of 16, so regions start 16-byte aligned), an upper bound on
its alignment width T (:458-459): for a subfamily
``max(pos + raw_len) - min(pos)`` (preprocessing only shortens reads and
never moves reference_start, :242-244); for a duplex the union of its two
subfamilies' bounds.
"""
from __future__ import annotations

import ctypes

import numpy as np

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_f64p = ctypes.POINTER(ctypes.c_double)


class DcrBatch(ctypes.Structure):
    _fields_ = [("n_fam", ctypes.c_int32), ("n_reads", ctypes.c_int32),
                ("n_cigar", ctypes.c_int64), ("n_bases", ctypes.c_int64),
                ("ss_cols", ctypes.c_int64), ("ds_cols", ctypes.c_int64),
                ("sub_off", ctypes.c_void_p), ("read_pos", ctypes.c_void_p),
                ("read_mapq", ctypes.c_void_p), ("seq_off", ctypes.c_void_p),
                ("seq_len", ctypes.c_void_p), ("cig_off", ctypes.c_void_p),
                ("cig_n", ctypes.c_void_p), ("cigar", ctypes.c_void_p),
                ("bases", ctypes.c_void_p), ("quals", ctypes.c_void_p),
                ("ss_col_off", ctypes.c_void_p), ("ds_col_off", ctypes.c_void_p)]


class DcrOut(ctypes.Structure):
    _fields_ = [("status", ctypes.c_void_p), ("pos", ctypes.c_void_p), ("mapq", ctypes.c_void_p),
                ("len", ctypes.c_void_p), ("n_cig", ctypes.c_void_p), ("n_de", ctypes.c_void_p),
                ("D", ctypes.c_void_p), ("M", ctypes.c_void_p), ("E", ctypes.c_void_p),
                ("seq", ctypes.c_void_p), ("qual", ctypes.c_void_p), ("cigar", ctypes.c_void_p),
                ("d", ctypes.c_void_p), ("e", ctypes.c_void_p)]


class DcrReadInfo(ctypes.Structure):
    _fields_ = [("seq_start", ctypes.c_int64), ("len", ctypes.c_int32), ("n_cig", ctypes.c_int32),
                ("status", ctypes.c_int32), ("has_ins", ctypes.c_int32)]


BATCH_FIELDS = ["sub_off", "read_pos", "read_mapq", "seq_off", "seq_len", "cig_off", "cig_n",
                "cigar", "bases", "quals", "ss_col_off", "ds_col_off"]
BATCH_DTYPES = dict(sub_off=np.int32, read_pos=np.int32, read_mapq=np.uint8, seq_off=np.int64,
                    seq_len=np.int32, cig_off=np.int32, cig_n=np.int32, cigar=np.uint32,
                    bases=np.uint8, quals=np.uint8, ss_col_off=np.int64, ds_col_off=np.int64)
OUT_SCALARS = dict(status=np.uint8, pos=np.int32, mapq=np.int32, len=np.int32, n_cig=np.int32,
                   n_de=np.int32, D=np.int32, M=np.int32, E=np.float64)
OUT_COLS = dict(seq=np.uint8, qual=np.uint8, cigar=np.uint32, d=np.uint16, e=np.uint16)


class PackedBatch:
    """numpy arrays of one batch (host memory)."""

    def __init__(self, **arrays):
        for k in BATCH_FIELDS:
            setattr(self, k, np.ascontiguousarray(arrays[k], dtype=BATCH_DTYPES[k]))
        self.n_fam = (len(self.sub_off) - 1) // 4
        self.n_reads = len(self.read_pos)

    @property
    def n_cigar(self):
        return len(self.cigar)

    @property
    def n_bases(self):
        return len(self.bases)

    @property
    def ss_cols(self):
        return int(self.ss_col_off[-1])

    @property
    def ds_cols(self):
        return int(self.ds_col_off[-1])

    def nbytes(self):
        return sum(getattr(self, k).nbytes for k in BATCH_FIELDS)

    def as_struct(self, ptrs=None) -> DcrBatch:
        """ctypes view; ``ptrs`` maps field -> device address (else host)."""
        s = DcrBatch()
        s.n_fam = self.n_fam
        s.n_reads = self.n_reads
        s.n_cigar = self.n_cigar
        s.n_bases = self.n_bases
        s.ss_cols = self.ss_cols
        s.ds_cols = self.ds_cols
        for k in BATCH_FIELDS:
            setattr(s, k, ptrs[k] if ptrs is not None else getattr(self, k).ctypes.data)
        return s


class OutArrays:
    """Host-side result arrays for one consensus kind."""

    def __init__(self, n_rec, n_cols):
        self.n_rec = n_rec
        for k, dt in OUT_SCALARS.items():
            setattr(self, k, np.zeros(n_rec, dtype=dt))
        for k, dt in OUT_COLS.items():
            setattr(self, k, np.zeros(max(n_cols, 1), dtype=dt))

    def as_struct(self, ptrs=None) -> DcrOut:
        s = DcrOut()
        for k in list(OUT_SCALARS) + list(OUT_COLS):
            setattr(s, k, ptrs[k] if ptrs is not None else getattr(self, k).ctypes.data)
        return s

    def record(self, i, col_off):
        """Decode consensus i into a plain dict (pos, mapq, cigar, seq, ...)."""
        b = int(col_off[i])
        n, nc, nd = int(self.len[i]), int(self.n_cig[i]), int(self.n_de[i])
        cig = self.cigar[b:b + nc]
        return dict(status=int(self.status[i]), pos=int(self.pos[i]), mapq=int(self.mapq[i]),
                    seq=self.seq[b:b + n].tobytes().decode(), qual=self.qual[b:b + n].tolist(),
                    cigar=[(int(c & 15), int(c >> 4)) for c in cig],
                    d=self.d[b:b + nd].tolist(), e=self.e[b:b + nd].tolist(),
                    D=int(self.D[i]), M=int(self.M[i]), E=float(self.E[i]))


def encode_cigar(cigartuples):
    return [(n << 4) | op for op, n in cigartuples]


def pack_families(families):
    """Pack families given as ``[A1, B2, B1, A2]`` lists of records (reads in
    reference order, already downsampled) into a PackedBatch."""
    reads = []
    sub_off = [0]
    for fam in families:
        assert len(fam) == 4
        for sub in fam:
            reads.extend(sub)
            sub_off.append(len(reads))
    n = len(reads)
    read_pos = np.empty(n, np.int32)
    read_mapq = np.empty(n, np.uint8)
    seq_len = np.empty(n, np.int32)
    cig_n = np.empty(n, np.int32)
    seqs, quals, cigs = [], [], []
    for i, r in enumerate(reads):
        read_pos[i] = r.reference_start
        read_mapq[i] = r.mapping_quality
        s = r.query_sequence or ""
        seq_len[i] = len(s)
        seqs.append(s.encode())
        q = r.query_qualities
        quals.append(bytes(q) if q is not None else b"\xff" * len(s))
        c = encode_cigar(r.cigartuples or [])
        cig_n[i] = len(c)
        cigs.extend(c)
    seq_off = np.zeros(n, np.int64)
    if n:
        seq_off[1:] = np.cumsum(seq_len[:-1], dtype=np.int64)
    cig_off = np.zeros(n, np.int32)
    if n:
        cig_off[1:] = np.cumsum(cig_n[:-1])
    bases = np.frombuffer(b"".join(seqs), np.uint8)
    qualv = np.frombuffer(b"".join(quals), np.uint8)
    return finish_batch(np.asarray(sub_off, np.int32), read_pos, read_mapq, seq_off, seq_len,
                        cig_off, cig_n, np.asarray(cigs, np.uint32), bases, qualv)


def _end_soft_clips(cigar, cig_off, cig_n):
    """Per read: length of the soft clip at the 5' end plus the one at the 3'
    end (each the first / last op, or the op inside a hard clip there)."""
    n = len(cig_n)
    out = np.zeros(n, np.int64)
    if n == 0 or len(cigar) == 0:
        return out
    cig = np.asarray(cigar, np.uint32)
    off = np.asarray(cig_off, np.int64)
    cn = np.asarray(cig_n, np.int64)
    has = cn > 0
    op = lambda i: (cig[np.clip(i, 0, len(cig) - 1)] & 15).astype(np.int64)
    ln = lambda i: (cig[np.clip(i, 0, len(cig) - 1)] >> 4).astype(np.int64)
    first, last = off, off + cn - 1
    c5 = np.where(op(first) == 4, ln(first), np.where((op(first) == 5) & (cn > 1) & (op(first + 1) == 4),
                                                      ln(first + 1), 0))
    i5 = np.where(op(first) == 4, first, first + 1)          # the op counted at the 5' end
    c3i = np.where(op(last) == 4, last, np.where((op(last) == 5) & (cn > 1), last - 1, -1))
    c3 = np.where((c3i >= first) & (op(c3i) == 4) & ~((c5 > 0) & (c3i == i5)), ln(c3i), 0)
    return np.where(has, c5 + c3, 0)


def _ranges(starts, lens):
    """Concatenated aranges [s, s + n) (vectorised)."""
    lens = lens.astype(np.int64)
    tot = int(lens.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    first = np.repeat(np.cumsum(lens) - lens, lens)
    return np.repeat(starts.astype(np.int64), lens) + (np.arange(tot, dtype=np.int64) - first)


def subset_families(packed: PackedBatch, fams) -> PackedBatch:
    """The batch of families ``fams`` (increasing indices) of ``packed``, in
    that order: a rank's share of a shared family stream."""
    fams = np.asarray(fams, np.int64)
    so = packed.sub_off.astype(np.int64)
    subs = (fams[:, None] * 4 + np.arange(4)[None, :]).reshape(-1)
    cnt = so[subs + 1] - so[subs]
    rd = _ranges(so[subs], cnt)
    sub_off = np.zeros(len(subs) + 1, np.int64)
    sub_off[1:] = np.cumsum(cnt)
    seq_len = packed.seq_len[rd]
    seq_off = np.zeros(len(rd), np.int64)
    seq_off[1:] = np.cumsum(seq_len[:-1].astype(np.int64))
    bi = _ranges(packed.seq_off[rd], seq_len)
    cig_n = packed.cig_n[rd]
    cig_off = np.zeros(len(rd), np.int64)
    cig_off[1:] = np.cumsum(cig_n[:-1].astype(np.int64))
    ci = _ranges(packed.cig_off[rd], cig_n)
    return finish_batch(sub_off, packed.read_pos[rd], packed.read_mapq[rd], seq_off, seq_len, cig_off, cig_n,
                        packed.cigar[ci], packed.bases[bi], packed.quals[bi])


def finish_batch(sub_off, read_pos, read_mapq, seq_off, seq_len, cig_off, cig_n, cigar, bases, quals):
    """Compute the output-region offsets (vectorised) and build the batch."""
    n_sub = len(sub_off) - 1
    F = n_sub // 4
    # kept length after remove_clipping (:191-265): a soft clip at either end
    # (inside a hard clip) drops its bases, so T below is the device's T before
    # the 3' N trim, exactly (regions are then exactly what the kernels fill)
    kept = seq_len.astype(np.int64) - _end_soft_clips(cigar, cig_off, cig_n)
    ends = read_pos.astype(np.int64) + kept
    cnt = np.diff(sub_off)
    if len(read_pos) and (cnt > 0).all():
        mn = np.minimum.reduceat(read_pos.astype(np.int64), sub_off[:-1])
        mx = np.maximum.reduceat(ends, sub_off[:-1])
    else:
        mn = np.zeros(n_sub, np.int64)
        mx = np.zeros(n_sub, np.int64)
        for s in range(n_sub):
            a, b = sub_off[s], sub_off[s + 1]
            if b > a:
                mn[s] = read_pos[a:b].min()
                mx[s] = ends[a:b].max()
    # regions are rounded up to 16 columns so every region starts 16-byte
    # aligned (the kernels write seq/qual/d/e with 16-byte stores)
    t_ss = (np.maximum(mx - mn, 1) + 15) & ~np.int64(15)
    ss_col_off = np.zeros(n_sub + 1, np.int64)
    ss_col_off[1:] = np.cumsum(t_ss)
    mn4, mx4 = mn.reshape(F, 4), mx.reshape(F, 4)
    t_ds = np.empty((F, 2), np.int64)
    for j, (a, b) in enumerate(((0, 1), (2, 3))):
        t_ds[:, j] = np.maximum(mx4[:, a], mx4[:, b]) - np.minimum(mn4[:, a], mn4[:, b])
    t_ds = (np.maximum(t_ds.reshape(-1), 1) + 15) & ~np.int64(15)
    ds_col_off = np.zeros(2 * F + 1, np.int64)
    ds_col_off[1:] = np.cumsum(t_ds)
    return PackedBatch(sub_off=sub_off, read_pos=read_pos, read_mapq=read_mapq, seq_off=seq_off,
                       seq_len=seq_len, cig_off=cig_off, cig_n=cig_n, cigar=cigar, bases=bases,
                       quals=quals, ss_col_off=ss_col_off, ds_col_off=ds_col_off)
