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


class DeviceStream:
    """Asynchronous batches on one GPU context (``_lib.Context``)."""

    def __init__(self, ctx, n_slots=2, owns_ctx=False):
        from . import _lib
        self.ctx = ctx
        self.owns_ctx = owns_ctx
        self.lib = _lib.load()
        self.n_slots = n_slots
        self.outs = [_HostOut(self.lib) for _ in range(n_slots)]
        self.busy = [False] * n_slots
        self.next_slot = 0
        self._pins = []

    def host_batch(self, reads=1 << 20):
        return native_io.HostBatch(reads=reads, alloc=pinned_allocator(self.lib, self._pins))

    def submit(self, hb):
        slot = self.next_slot
        self.next_slot = (slot + 1) % self.n_slots
        if self.busy[slot]:
            raise RuntimeError("DeviceStream: slot reused before its result was taken")
        s = hb.s
        out = self.outs[slot]
        out.ensure(4 * s.n_fam, s.ss_cols, 2 * s.n_fam, s.ds_cols, s.n_reads)
        self._b = hb.batch_struct()
        so, do = out.dcr_out("ss"), out.dcr_out("ds")
        from . import _lib
        _lib._check(self.lib.dcr_submit(self.ctx._ctx, slot, ctypes.byref(self._b), ctypes.byref(so),
                                        ctypes.byref(do), out.arr["rs"]["status"].ctypes.data))
        self.busy[slot] = True
        return slot

    def result(self, slot):
        from . import _lib
        _lib._check(self.lib.dcr_wait(self.ctx._ctx, slot))
        self.busy[slot] = False
        out = self.outs[slot]
        return out.fmt_out("ss"), out.fmt_out("ds"), out.arr["rs"]["status"]

    def close(self):
        for slot in range(self.n_slots):
            if self.busy[slot]:
                self.lib.dcr_wait(self.ctx._ctx, slot)
                self.busy[slot] = False
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
