"""Batch backends for the streaming driver (cli.py).

``DeviceStream`` is the product path: host batches live in pinned memory
(``dcr_host_alloc``), each ``submit`` is one asynchronous ``dcr_submit``
(H2D on a copy stream, the kernels on the compute stream, D2H of the fields
the writer needs on a second copy stream) and ``result`` waits for that
slot only, so the ingest of batch k+1 and the writing of batch k-1 overlap
the device work of batch k (north_star: "a writer that streams results back
through hipMemcpyAsync on side streams").

``CallBackend`` wraps a synchronous ``(packed, params) -> (ss, ds, info)``
callable (the C oracle in CPU tests, test infrastructure only).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native_io
from .batch import DcrOut, OUT_COLS, OUT_SCALARS

# fields of the single-strand results the writer reads (dcr_fmt_out); pos,
# n_cig and cigar of single-strand records stay on the device
SS_FIELDS = ("status", "mapq", "len", "n_de", "D", "M", "E", "seq", "qual", "d", "e")
DS_FIELDS = tuple(OUT_SCALARS) + tuple(OUT_COLS)


class Pinned:
    """A pinned host allocation (hipHostMalloc) viewed as a uint8 numpy array."""

    def __init__(self, lib, nbytes):
        self._lib = lib
        self.nbytes = max(int(nbytes), 16)
        self.ptr = lib.dcr_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"dcr_host_alloc({self.nbytes}) failed")
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self._lib.dcr_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def pinned_allocator(lib, keep):
    def alloc(nbytes):
        p = Pinned(lib, nbytes)
        keep.append(p)
        return p.array
    return alloc


class _HostOut:
    """Pinned host arrays receiving one slot's outputs (grow-only)."""

    def __init__(self, lib):
        self.lib = lib
        self.cap = None
        self.mem = None
        self.arr = {}

    def ensure(self, n_ss, c_ss, n_ds, c_ds, n_reads):
        need = (n_ss, c_ss, n_ds, c_ds, n_reads)
        if self.cap is not None and all(a >= b for a, b in zip(self.cap, need)):
            return
        cap = tuple(int(max(b, 1) * 1.25) + 64 for b in need)
        specs = []
        for kind, fields, nrec, ncol in (("ss", SS_FIELDS, cap[0], cap[1]), ("ds", DS_FIELDS, cap[2], cap[3])):
            for k in fields:
                dt = OUT_SCALARS.get(k) or OUT_COLS[k]
                specs.append((kind, k, np.dtype(dt), nrec if k in OUT_SCALARS else ncol))
        specs.append(("rs", "status", np.dtype(np.int32), cap[4]))
        total = sum(((dt.itemsize * n + 255) & ~255) for _, _, dt, n in specs)
        if self.mem is not None:
            self.mem.free()
        self.mem = Pinned(self.lib, total)
        self.arr = {"ss": {}, "ds": {}, "rs": {}}
        off = 0
        for kind, k, dt, n in specs:
            self.arr[kind][k] = self.mem.array[off:off + dt.itemsize * n].view(dt)
            off += (dt.itemsize * n + 255) & ~255
        self.cap = cap

    def dcr_out(self, kind):
        o = DcrOut()
        for k, _ in DcrOut._fields_:
            a = self.arr[kind].get(k)
            setattr(o, k, a.ctypes.data if a is not None else None)
        return o

    def fmt_out(self, kind):
        o = native_io.FmtOut()
        for k, _ in native_io.FmtOut._fields_:
            a = self.arr[kind].get(k)
            setattr(o, k, a.ctypes.data if a is not None else None)
        return o


class WMeta(ctypes.Structure):
    _fields_ = [("names", ctypes.c_void_p), ("n_names", ctypes.c_int64), ("fam_code", ctypes.c_void_p),
                ("fam_rx", ctypes.c_void_p), ("fam_tid", ctypes.c_void_p)]


class WRes(ctypes.Structure):
    _fields_ = [("bgzf", ctypes.c_void_p), ("cap_bgzf", ctypes.c_int64), ("fam_fail", ctypes.c_void_p),
                ("ds_len", ctypes.c_void_p), ("totals", ctypes.c_void_p)]


class _WriterOut:
    """Pinned host arrays of one slot's device-writer results (grow-only)."""

    def __init__(self, lib):
        self.lib = lib
        self.cap_f = 0
        self.cap_b = 0
        self.small = None
        self.blocks = None

    def ensure(self, n_fam, bgzf_bytes):
        if n_fam > self.cap_f or self.small is None:
            self.cap_f = int(n_fam * 1.25) + 64
            self.small = Pinned(self.lib, 12 * self.cap_f + 64)
            a = self.small.array
            self.fam_fail = a[:4 * self.cap_f].view(np.int32)
            self.ds_len = a[4 * self.cap_f:12 * self.cap_f].view(np.int32)
            self.totals = a[12 * self.cap_f:12 * self.cap_f + 24].view(np.int64)
        if bgzf_bytes > self.cap_b:
            self.cap_b = int(bgzf_bytes * 1.25) + (1 << 20)
            self.blocks = Pinned(self.lib, self.cap_b)

    def wres(self):
        r = WRes()
        r.bgzf, r.cap_bgzf = self.blocks.ptr, self.cap_b
        r.fam_fail, r.ds_len, r.totals = self.fam_fail.ctypes.data, self.ds_len.ctypes.data, self.totals.ctypes.data
        return r


class WriterResult:
    """One batch through the device writer: per-family outcomes (0: written),
    duplex lengths, and the BGZF blocks of the records of every family that
    does not fail."""

    def __init__(self, stream, slot, out, n_fam):
        self._stream, self._slot = stream, slot
        self.fam_fail = out.fam_fail[:n_fam]
        self.ds_len = out.ds_len[:2 * n_fam]
        self.bgzf_bytes, self.record_bytes, self.blocks = (int(x) for x in out.totals[:3])
        self.bgzf = out.blocks.array[:self.bgzf_bytes]

    def record_bytes_of(self, n_fam):
        """Formatted records of families [0, n_fam) (fetched from the device slot)."""
        lib, ctx = self._stream.lib, self._stream.ctx._ctx
        from . import _lib
        end = np.zeros(1, np.int64)
        _lib._check(lib.dcr_slot_fetch(ctx, self._slot, 1, 2 * n_fam, 1, end.ctypes.data))
        buf = np.zeros(max(int(end[0]), 1), np.uint8)
        _lib._check(lib.dcr_slot_fetch(ctx, self._slot, 0, 0, int(end[0]), buf.ctypes.data))
        return buf[:int(end[0])]


class DeviceStream:
    """Asynchronous batches on one GPU context (``_lib.Context``).  With
    ``device_writer`` the records are formatted and BGZF-compressed on the
    device (dcr_submit_write); otherwise the kernel outputs come back for the
    host writer (dcr_submit)."""

    def __init__(self, ctx, n_slots=2, owns_ctx=False, device_writer=True, persistent=False):
        """``persistent``: ``close`` only drains the slots (the context and the
        released host batches stay for the next run, cli.default_backend);
        ``close(final=True)`` frees them."""
        from . import _lib
        self.ctx = ctx
        self.owns_ctx = owns_ctx
        self.persistent = persistent
        self.closed = False
        self._spare = {}                 # reads -> [HostBatch] released by earlier runs
        self.device_writer = device_writer
        self.lib = _lib.load()
        self.n_slots = n_slots
        self.outs = [_HostOut(self.lib) for _ in range(n_slots)]
        self.wouts = [_WriterOut(self.lib) for _ in range(n_slots)]
        self.busy = [False] * n_slots
        self.next_slot = 0
        self._pins = []

    def host_batch(self, reads=1 << 20):
        spare = self._spare.get(reads)
        if spare:
            return spare.pop()
        return native_io.HostBatch(reads=reads, alloc=pinned_allocator(self.lib, self._pins))

    def release(self, batches):
        """Host batches a run is done with, kept for the next run (persistent)."""
        if self.persistent and not self.closed:
            for hb in batches:
                self._spare.setdefault(hb.reads, []).append(hb)

    def submit(self, hb):
        slot = self.next_slot
        self.next_slot = (slot + 1) % self.n_slots
        if self.busy[slot]:
            raise RuntimeError("DeviceStream: slot reused before its result was taken")
        s = hb.s
        if self.device_writer:
            from . import _lib
            wo = self.wouts[slot]
            # compressed records are far smaller than the kernel outputs; grown on demand
            wo.ensure(s.n_fam, max(64 << 20, 2 * s.n_bases // 3))
            self._b = hb.batch_struct()
            m = WMeta()
            m.names, m.n_names = hb.a["names"].ctypes.data, s.n_names
            m.fam_code, m.fam_rx, m.fam_tid = (hb.a["fam_code"].ctypes.data, hb.a["fam_rx"].ctypes.data,
                                               hb.a["fam_tid"].ctypes.data)
            self._wres = wo.wres()
            _lib._check(self.lib.dcr_submit_write(self.ctx._ctx, slot, ctypes.byref(self._b), ctypes.byref(m),
                                                  ctypes.byref(self._wres)))
            self.busy[slot] = True
            return (slot, s.n_fam)
        out = self.outs[slot]
        out.ensure(4 * s.n_fam, s.ss_cols, 2 * s.n_fam, s.ds_cols, s.n_reads)
        self._b = hb.batch_struct()
        so, do = out.dcr_out("ss"), out.dcr_out("ds")
        from . import _lib
        _lib._check(self.lib.dcr_submit(self.ctx._ctx, slot, ctypes.byref(self._b), ctypes.byref(so),
                                        ctypes.byref(do), None))
        self.busy[slot] = True
        return slot

    def result(self, handle):
        from . import _lib
        if self.device_writer:
            slot, n_fam = handle
            wo = self.wouts[slot]
            r = wo.wres()
            rc = self.lib.dcr_wait_write(self.ctx._ctx, slot, ctypes.byref(r))
            self.busy[slot] = False
            if rc == 3 and int(wo.totals[0]) > wo.cap_b:      # DCR_ECAPACITY: grow, fetch again
                n = int(wo.totals[0])
                tot = wo.totals[:3].copy()
                wo.ensure(n_fam, n)
                wo.totals[:3] = tot
                _lib._check(self.lib.dcr_slot_fetch(self.ctx._ctx, slot, 2, 0, n, wo.blocks.ptr))
            else:
                _lib._check(rc)
            return WriterResult(self, slot, wo, n_fam)
        slot = handle
        _lib._check(self.lib.dcr_wait(self.ctx._ctx, slot))
        self.busy[slot] = False
        out = self.outs[slot]
        return out.fmt_out("ss"), out.fmt_out("ds"), None

    def close(self, final=False):
        if self.closed:
            return
        for slot in range(self.n_slots):
            if self.busy[slot]:
                if self.device_writer:
                    self.lib.dcr_wait_write(self.ctx._ctx, slot, ctypes.byref(self.wouts[slot].wres()))
                else:
                    self.lib.dcr_wait(self.ctx._ctx, slot)
                self.busy[slot] = False
        if self.persistent and not final:
            return
        self.closed = True
        self._spare.clear()
        for p in self._pins:
            p.free()
        self._pins.clear()
        for o in self.outs:
            if o.mem is not None:
                o.mem.free()
        for w in self.wouts:
            for m in (w.small, w.blocks):
                if m is not None:
                    m.free()
        if self.owns_ctx:
            self.ctx.close()


class CallBackend:
    """Synchronous backend over ``fn(packed, params) -> (ss, ds, info)``."""

    def __init__(self, fn, params):
        self.fn, self.params = fn, params
        self._res = {}
        self._k = 0

    def host_batch(self, reads=1 << 20):
        return native_io.HostBatch(reads=reads)

    def submit(self, hb):
        ss, ds, info = self.fn(hb.packed(), self.params)
        self._k += 1
        rs = None if info is None else np.ascontiguousarray(info["status"], np.int32)
        self._res[self._k] = (ss, ds, rs)
        return self._k

    def result(self, h):
        ss, ds, rs = self._res.pop(h)
        self._keep = (ss, ds, rs)
        return native_io.fmt_out(ss), native_io.fmt_out(ds), rs

    def close(self):
        self._res.clear()
