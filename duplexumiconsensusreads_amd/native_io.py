"""ctypes binding of libdcr_io.so (include/dcr_io.h): native BAM ingest into
packed batches, the consensus record writer and the BGZF writer.

These replace the per-record Python host work around the kernels (the
reference's streaming loop over pysam, DuplexUMIConsensusReads.py:1519-1594):
the Python side only moves whole batches between the ingest, the device and
the writer.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .batch import BATCH_FIELDS, BATCH_DTYPES, DcrBatch, PackedBatch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DCR_IO_LIB", os.path.join(HERE, "libdcr_io.so"))   # DCR_IO_LIB: A/B builds (tools/)

_i32, _i64, _vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p

END_FULL, END_EOF, END_ERROR = 0, 1, 2
INGEST_HOST_INFLATE = 1                  # dcr_ingest_cfg.flags
ERR_NAMES = {1: "exit", 2: "TypeError", 3: "IndexError", 4: "ValueError", 5: "AttributeError"}
FAM_PROCESSED, FAM_FILTERED = 0, 1
FAIL_NAMES = {1: "IndexError", 2: "TypeError", 3: "ValueError", 4: "OverflowError", 5: "exit",
              7: "UnicodeEncodeError"}


class IngestCfg(ctypes.Structure):
    _fields_ = [("min_map_quality", _i32), ("min_reads", _i32), ("max_reads", _i32),
                ("min_base_quality", _i32), ("n_threads", _i32), ("flags", _i32)]


# (name, dtype, length expression) of the caller-owned arrays, in struct order
_HB_ARRAYS = [
    ("sub_off", np.int32, "4f1"), ("read_pos", np.int32, "r"), ("read_mapq", np.uint8, "r"),
    ("seq_off", np.int64, "r"), ("seq_len", np.int32, "r"), ("cig_off", np.int32, "r"),
    ("cig_n", np.int32, "r"), ("cigar", np.uint32, "c"), ("bases", np.uint8, "b"), ("quals", np.uint8, "b"),
    ("ss_col_off", np.int64, "4f1"), ("ds_col_off", np.int64, "2f1"),
    ("fam_tid", np.int32, "f"), ("fam_code", np.int64, "f"), ("fam_rx", np.int64, "2f"),
    ("fam_eqx", np.uint16, "4f"),
    ("tab_kind", np.int32, "t"), ("tab_proc", np.int32, "t"), ("tab_sampled", np.int32, "t"),
    ("tab_code", np.int64, "t"), ("tab_exc_cut", np.int64, "t"), ("tab_filt_cut", np.int64, "t"),
    ("names", np.uint8, "n"), ("side_exc", np.uint8, "s"), ("side_filt", np.uint8, "s"),
]


class HostBatchStruct(ctypes.Structure):
    _fields_ = ([("cap_fam", _i32), ("cap_tab", _i32), ("cap_reads", _i32), ("reserved0", _i32),
                 ("cap_cigar", _i64), ("cap_bases", _i64), ("cap_names", _i64), ("cap_side", _i64)]
                + [(n, _vp) for n, _, _ in _HB_ARRAYS]
                + [("n_fam", _i32), ("n_reads", _i32), ("n_cigar", _i64), ("n_bases", _i64),
                   ("ss_cols", _i64), ("ds_cols", _i64), ("n_tab", _i32), ("end_kind", _i32),
                   ("n_names", _i64), ("n_side_exc", _i64), ("n_side_filt", _i64),
                   ("err_kind", _i32), ("reserved1", _i32), ("err_msg", ctypes.c_char * 512)])


class SynthIn(ctypes.Structure):
    _fields_ = [("n_fam", _i32), ("tid", _i32), ("fam_id0", _i64)] + [
        (n, _vp) for n in ("sub_off", "read_pos", "read_mapq", "seq_off", "seq_len", "cig_off", "cig_n", "cigar",
                           "bases", "quals", "umis")]


class FmtOut(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("status", "pos", "mapq", "len", "n_cig", "n_de", "D", "M", "E", "seq", "qual",
                                   "cigar", "d", "e")]


_lib = None


class IOError_(RuntimeError):
    pass


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise IOError_(f"{LIB_PATH} not built - run __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        sig = {
            "dcr_io_abi_version": (_i32, []),
            "dcr_io_last_error": (ctypes.c_char_p, []),
            "dcr_ingest_open": (_vp, [ctypes.c_char_p, _vp]),
            "dcr_ingest_close": (None, [_vp]),
            "dcr_ingest_header": (_i64, [_vp, ctypes.POINTER(_vp)]),
            "dcr_ingest_set_rng": (_i32, [_vp, _vp, _i32]),
            "dcr_ingest_get_rng": (_i32, [_vp, _vp, _vp]),
            "dcr_ingest_next": (_i32, [_vp, _vp]),
            "dcr_ingest_counters": (_i32, [_vp, _vp]),
            "dcr_py_sample": (_i32, [_vp, _vp, _i32, _i32, _vp]),
            "dcr_bgzw_open": (_vp, [ctypes.c_char_p, _i32, _i32]),
            "dcr_bgzw_write": (_i32, [_vp, _vp, _i64]),
            "dcr_bgzw_close": (_i32, [_vp]),
            "dcr_bgzw_put_blocks": (_i32, [_vp, _vp, _i64, _i64]),
            "dcr_bgzw_sizes": (_i32, [_vp, _vp]),
            "dcr_fmt_scan": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _vp]),
            "dcr_fmt_write": (_i32, [_vp, _vp, _vp, _vp, _i32]),
            "dcr_synth_write": (_i32, [_vp, _vp, _i32]),
            "dcr_deflate_emulate": (_i64, [_vp, _i64, _vp]),
            "dcr_deflate_lengths_ab": (_i32, [_vp, _i32, _vp, _vp]),
            "dcr_split_points": (_i32, [ctypes.c_char_p, _i32, _vp, _vp]),
            "dcr_ingest_open_range": (_vp, [ctypes.c_char_p, _vp, _i64, _i64]),
            "dcr_ingest_sample_calls": (_i64, [_vp, _vp, _i64]),
            "dcr_py_replay": (_i32, [_vp, _vp, _vp, _i64]),
            "dcr_bam_header": (_i64, [ctypes.c_char_p, _vp, _i64]),
            "dcr_io_set_inflate_hook": (_i32, [_vp]),
            "dcr_ingest_gpu_inflate": (_i32, [_vp]),
            "dcr_ingest_set_state_gate": (_i32, [_vp, _vp, _vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dcr_io_abi_version() != 1:
            raise IOError_("libdcr_io.so ABI mismatch")
        _lib = lib
    return _lib


def _err(what):
    return IOError_(f"{what}: {load().dcr_io_last_error().decode(errors='replace')}")


def numpy_alloc(nbytes):
    return np.zeros(max(nbytes, 1), np.uint8)


class HostBatch:
    """One batch's caller-owned arrays (``dcr_host_batch``), carved from a
    single allocation (``alloc(nbytes) -> uint8 array``; pinned host memory
    on the GPU path)."""

    def __init__(self, reads=1 << 20, avg_len=160, side_bytes=64 << 20, alloc=numpy_alloc):
        self.reads = reads
        # a processed family holds at least one read per subfamily (min_reads
        # >= 1); a batch simply ends early when a table fills first
        f = max(reads // 4 + 16, 16)
        t = 2 * f
        caps = {"r": reads, "f": f, "4f": 4 * f, "4f1": 4 * f + 1, "2f": 2 * f, "2f1": 2 * f + 1, "t": t,
                "c": 8 * reads, "b": avg_len * reads, "n": 96 * t + (1 << 16), "s": side_bytes}
        # pinned: what crosses PCIe (the dcr_batch arrays and the writer's
        # metadata); the family table and the side-file records stay host-only
        host_only = {"side_exc", "side_filt", "tab_kind", "tab_proc", "tab_sampled", "tab_code", "tab_exc_cut",
                     "tab_filt_cut"}
        lay, off = [], 0
        for name, dt, ln in _HB_ARRAYS:
            if name in host_only:
                continue
            nb = np.dtype(dt).itemsize * caps[ln]
            off = (off + 255) & ~255
            lay.append((name, dt, off, caps[ln]))
            off += nb
        self.mem = alloc(off)
        s = HostBatchStruct()
        s.cap_fam, s.cap_tab, s.cap_reads = f, t, reads
        s.cap_cigar, s.cap_bases, s.cap_names, s.cap_side = caps["c"], caps["b"], caps["n"], caps["s"]
        self.a = {}
        base = self.mem.ctypes.data
        for name, dt, o, n in lay:
            self.a[name] = self.mem[o:o + n * np.dtype(dt).itemsize].view(dt)
            setattr(s, name, base + o)
        for name, dt, ln in _HB_ARRAYS:
            if name in host_only:                   # ordinary (lazily paged) memory
                self.a[name] = np.empty(caps[ln], dt)
                setattr(s, name, self.a[name].ctypes.data)
        self.s = s

    # -- filled fields ---------------------------------------------------------
    @property
    def n_fam(self):
        return self.s.n_fam

    @property
    def end_kind(self):
        return self.s.end_kind

    def packed(self) -> PackedBatch:
        """numpy views of the dcr_batch part (no copies)."""
        s = self.s
        F, n = s.n_fam, s.n_reads
        lens = {"sub_off": 4 * F + 1, "read_pos": n, "read_mapq": n, "seq_off": n, "seq_len": n, "cig_off": n,
                "cig_n": n, "cigar": s.n_cigar, "bases": s.n_bases, "quals": s.n_bases,
                "ss_col_off": 4 * F + 1, "ds_col_off": 2 * F + 1}
        pb = PackedBatch.__new__(PackedBatch)
        for k in BATCH_FIELDS:
            setattr(pb, k, self.a[k][:lens[k]])
        pb.n_fam, pb.n_reads = F, n
        return pb

    def batch_struct(self) -> DcrBatch:
        s = self.s
        b = DcrBatch()
        b.n_fam, b.n_reads, b.n_cigar, b.n_bases = s.n_fam, s.n_reads, s.n_cigar, s.n_bases
        b.ss_cols, b.ds_cols = s.ss_cols, s.ds_cols
        for k in BATCH_FIELDS:
            setattr(b, k, self.a[k].ctypes.data)
        return b

    def name(self, off):
        nm = self.a["names"]
        e = int(off)
        while nm[e] != 0:
            e += 1
        return nm[int(off):e].tobytes().decode("latin-1")

    def table(self):
        """[(kind, processed index, sampled mask, code, exc_cut, filt_cut)] in input order."""
        s, a = self.s, self.a
        return [(int(a["tab_kind"][t]), int(a["tab_proc"][t]), int(a["tab_sampled"][t]), self.name(a["tab_code"][t]),
                 int(a["tab_exc_cut"][t]), int(a["tab_filt_cut"][t])) for t in range(s.n_tab)]

    def side(self, which):
        n = self.s.n_side_exc if which == "exc" else self.s.n_side_filt
        return self.a["side_exc" if which == "exc" else "side_filt"][:n]

    def error(self):
        return ERR_NAMES.get(self.s.err_kind), self.s.err_msg.decode(errors="replace")


_HOOK = None    # the dcr_inflate_hook passed to the library (kept alive here)


def set_inflate_hook(hook):
    """Ingests opened after this inflate their BGZF members with ``hook``
    (a ``_lib.InflateHook`` from ``_lib.Inflater.hook()``: the device
    inflater); None goes back to the host pool (dcr_io_set_inflate_hook)."""
    global _HOOK
    if load().dcr_io_set_inflate_hook(ctypes.byref(hook) if hook is not None else None) != 0:
        raise _err("set_inflate_hook")
    _HOOK = hook


_GATE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                            ctypes.POINTER(ctypes.c_int32))


class Ingest:
    """dcr_ingest: a BAM opened for batched reading."""

    def __init__(self, path, min_map_quality=20, min_reads=1, max_reads=100, min_base_quality=20, n_threads=0,
                 start_voff=0, end_voff=-1, host_inflate=False):
        """``start_voff`` / ``end_voff``: a range of whole families
        (split_points); the header is then empty.  ``host_inflate``: the host
        inflate pool even when a GPU inflate hook is set."""
        lib = load()
        cfg = IngestCfg(min_map_quality, min_reads, max_reads, min_base_quality, n_threads,
                        INGEST_HOST_INFLATE if host_inflate else 0)
        if start_voff == 0 and end_voff == -1:
            self._h = lib.dcr_ingest_open(os.fsencode(path), ctypes.byref(cfg))
        else:
            self._h = lib.dcr_ingest_open_range(os.fsencode(path), ctypes.byref(cfg), int(start_voff), int(end_voff))
        if not self._h:
            raise _err(f"cannot read {path}")
        p = _vp()
        n = lib.dcr_ingest_header(self._h, ctypes.byref(p))
        self.header = ctypes.string_at(p.value, n) if n > 0 else b""

    @property
    def gpu_inflate(self) -> bool:
        """True when this ingest inflates on the GPU (set_inflate_hook)."""
        return bool(load().dcr_ingest_gpu_inflate(self._h))

    def sample_calls(self):
        """(population, sample size) of every random.sample call so far."""
        lib = load()
        n = lib.dcr_ingest_sample_calls(self._h, None, 0)
        out = np.zeros(2 * max(n, 1), np.int32)
        lib.dcr_ingest_sample_calls(self._h, out.ctypes.data, n)
        return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]

    def set_rng_state(self, state):
        """``random.getstate()`` of a CPython generator."""
        words = np.asarray(state[1][:624], np.uint32)
        if load().dcr_ingest_set_rng(self._h, words.ctypes.data, int(state[1][624])) != 0:
            raise _err("set_rng")

    def set_state_gate(self, fn):
        """``fn()`` -> a ``random.getstate()`` tuple, called once on the thread
        running next(), right before this ingest's first random.sample call
        (never when it does not sample); None removes the gate.  An exception
        in ``fn`` ends the ingest with an error."""
        lib = load()
        if fn is None:
            self._gate = None
            lib.dcr_ingest_set_state_gate(self._h, None, None)
            return

        def gate(_user, mt, index):
            try:
                st = fn()
                words = np.asarray(st[1][:624], np.uint32)
                ctypes.memmove(mt, words.ctypes.data, 624 * 4)
                index[0] = int(st[1][624])
                return 0
            except BaseException as e:   # noqa: BLE001 - reported through the ingest's error
                self.gate_error = e
                return 1
        self.gate_error = None
        self._gate = _GATE_FN(gate)      # kept alive with the ingest
        if lib.dcr_ingest_set_state_gate(self._h, ctypes.cast(self._gate, _vp), None) != 0:
            raise _err("set_state_gate")

    def rng_state(self, template):
        words = np.zeros(624, np.uint32)
        idx = ctypes.c_int32()
        if load().dcr_ingest_get_rng(self._h, words.ctypes.data, ctypes.byref(idx)) != 0:
            raise _err("get_rng")
        return (template[0], tuple(int(x) for x in words) + (idx.value,), template[2])

    def next(self, hb: HostBatch) -> HostBatch:
        rc = load().dcr_ingest_next(self._h, ctypes.byref(hb.s))
        if rc != 0:
            raise _err("ingest")
        return hb

    def counters(self):
        out = np.zeros(5, np.int64)
        load().dcr_ingest_counters(self._h, out.ctypes.data)
        return dict(passed=int(out[0]), excluded=int(out[1]), processed=int(out[2]), filtered=int(out[3]),
                    records=int(out[4]))

    def close(self):
        if getattr(self, "_h", None):
            load().dcr_ingest_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BgzfWriter:
    """dcr_bgzw: BGZF output (libdeflate blocks on a pool)."""

    def __init__(self, path, header: bytes, level=6, n_threads=0):
        lib = load()
        self._h = lib.dcr_bgzw_open(os.fsencode(path), level, n_threads)
        if not self._h:
            raise _err(f"cannot write {path}")
        try:
            self.write(header)
        except BaseException:
            lib.dcr_bgzw_close(self._h)
            self._h = None
            raise

    def write(self, data):
        if isinstance(data, np.ndarray):
            ptr, n = data.ctypes.data, data.nbytes
        else:
            buf = ctypes.create_string_buffer(bytes(data), len(data))
            ptr, n = ctypes.addressof(buf), len(data)
        if n and load().dcr_bgzw_write(self._h, ptr, n) != 0:
            raise _err("BGZF write")

    def put_blocks(self, blocks: np.ndarray, raw_bytes: int):
        """Append BGZF blocks compressed elsewhere (the device writer)."""
        if load().dcr_bgzw_put_blocks(self._h, blocks.ctypes.data, blocks.nbytes, raw_bytes) != 0:
            raise _err("BGZF put_blocks")

    def write_consensus(self, hb: HostBatch, ss: FmtOut, ds: FmtOut, n_fam: int):
        if n_fam and load().dcr_fmt_write(self._h, ctypes.byref(hb.s), ctypes.byref(ss), ctypes.byref(ds),
                                          n_fam) != 0:
            raise _err("consensus write")

    def write_synthetic(self, packed, umis, fam_id0=0, tid=0, n_threads=0):
        """Records of every family of ``packed`` (dcr_synth_write)."""
        si = SynthIn()
        si.n_fam, si.tid, si.fam_id0 = packed.n_fam, tid, fam_id0
        for k in ("sub_off", "read_pos", "read_mapq", "seq_off", "seq_len", "cig_off", "cig_n", "cigar", "bases",
                  "quals"):
            setattr(si, k, getattr(packed, k).ctypes.data)
        u = np.ascontiguousarray(umis, dtype=np.uint8)
        assert u.size >= 16 * packed.n_fam
        si.umis = u.ctypes.data
        if load().dcr_synth_write(self._h, ctypes.byref(si), n_threads) != 0:
            raise _err("synthetic write")

    def sizes(self):
        out = np.zeros(2, np.int64)
        load().dcr_bgzw_sizes(self._h, out.ctypes.data)
        return int(out[0]), int(out[1])

    def close(self):
        if getattr(self, "_h", None):
            rc = load().dcr_bgzw_close(self._h)
            self._h = None
            if rc != 0:
                raise _err("BGZF close")


def fmt_out(arrays) -> FmtOut:
    """FmtOut over host result arrays (batch.OutArrays, or a dict of arrays)."""
    o = FmtOut()
    for k, _ in FmtOut._fields_:
        v = arrays[k] if isinstance(arrays, dict) else getattr(arrays, k)
        setattr(o, k, v.ctypes.data if isinstance(v, np.ndarray) else int(v))
    return o


def first_failure(hb: HostBatch, ss: FmtOut, ds: FmtOut, n_fam: int, read_status=None):
    """(index of the first failing processed family or n_fam, exception name, which consensus)."""
    kind, which = ctypes.c_int32(), ctypes.c_int32()
    rs = read_status.ctypes.data if read_status is not None else None
    f = load().dcr_fmt_scan(ctypes.byref(hb.s), ctypes.byref(ss), ctypes.byref(ds), rs, n_fam,
                            ctypes.byref(kind), ctypes.byref(which))
    return f, FAIL_NAMES.get(kind.value), which.value


def deflate_emulate(data: bytes) -> bytes:
    """One BGZF block from the GPU compressor's algorithm, emulated on the host."""
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    out = ctypes.create_string_buffer(65536)
    n = load().dcr_deflate_emulate(buf, len(data), out)
    if n < 0:
        raise IOError_("deflate_emulate: bad input size")
    return out.raw[:n]


def split_points(path, n_parts, params):
    """dcr_split_points: BGZF virtual offsets where parts 1..n-1 of the input
    start (each a family start), -1 where none was found."""
    cfg = IngestCfg(params.min_map_quality, params.min_reads, params.max_reads, params.min_base_quality, 0, 0)
    out = np.full(max(n_parts - 1, 1), -1, np.int64)
    if load().dcr_split_points(os.fsencode(path), n_parts, ctypes.byref(cfg), out.ctypes.data) != 0:
        raise _err("split_points")
    return [int(v) for v in out[:n_parts - 1]]


def bam_header(path):
    """The BAM header as stored (dcr_bam_header)."""
    lib = load()
    n = lib.dcr_bam_header(os.fsencode(path), None, 0)
    if n < 0:
        raise _err(f"cannot read {path}")
    buf = ctypes.create_string_buffer(n)
    lib.dcr_bam_header(os.fsencode(path), buf, n)
    return buf.raw[:n]


def py_replay(state, calls):
    """A CPython random state after random.sample(range(n), k) for each (n, k)."""
    words = np.asarray(state[1][:624], np.uint32).copy()
    index = ctypes.c_int32(int(state[1][624]))
    c = np.asarray(calls, np.int32).reshape(-1)
    if load().dcr_py_replay(words.ctypes.data, ctypes.byref(index), c.ctypes.data if c.size else None,
                            len(calls)) != 0:
        raise _err("py_replay")
    return (state[0], tuple(int(w) for w in words) + (int(index.value),), state[2])


def py_sample(state, n, k):
    """CPython random.sample(range(n), k) through the native MT19937 (tests)."""
    words = np.asarray(state[1][:624], np.uint32).copy()
    idx = ctypes.c_int32(int(state[1][624]))
    out = np.zeros(max(k, 1), np.int32)
    if load().dcr_py_sample(words.ctypes.data, ctypes.byref(idx), n, k, out.ctypes.data) != 0:
        raise _err("sample")
    return out[:k].tolist(), (state[0], tuple(int(x) for x in words) + (idx.value,), state[2])
