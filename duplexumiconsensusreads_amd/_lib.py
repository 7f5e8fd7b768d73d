"""ctypes binding of libdcr.so (the C-ABI in include/dcr.h).

This is the product path: it loads the in-tree HIP library built for gfx950
and fails loudly if it is missing or the device is not an MI355X.  There is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .batch import DcrBatch, DcrOut, DcrReadInfo, OutArrays, PackedBatch
from .params import ConsensusParams, DcrParams, build_dcr_params

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DCR_LIB", os.path.join(HERE, "libdcr.so"))

EXPORTS = {
    "dcr_abi_version": (ctypes.c_int, []),
    "dcr_last_error": (ctypes.c_char_p, []),
    "dcr_create": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_void_p]),
    "dcr_destroy": (None, [ctypes.c_void_p]),
    "dcr_set_params": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_set_options": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "dcr_reserve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "dcr_run_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_run_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "dcr_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "dcr_read_info_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "dcr_last_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_last_kernel_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_host_alloc": (ctypes.c_void_p, [ctypes.c_size_t]),
    "dcr_host_free": (None, [ctypes.c_void_p]),
    "dcr_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p]),
    "dcr_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "dcr_submit_write": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "dcr_wait_write": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "dcr_slot_fetch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_void_p]),
    # include/dcr_inflate.h: BGZF inflate on the device
    "dcr_inflater_create": (ctypes.c_void_p, [ctypes.c_int]),
    "dcr_inflater_destroy": (None, [ctypes.c_void_p]),
    "dcr_inflater_hook": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_inflater_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64]),
    "dcr_inflater_last": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_inflater_totals": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "dcr_inflate_stream_open": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_void_p]),
    "dcr_inflate_stream_add": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]),
    "dcr_inflate_stream_fetch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]),
    "dcr_inflate_stream_close": (None, [ctypes.c_void_p]),
}

# HIP-event slots of dcr_last_kernel_timing: k_recmeta<ss> includes k_prep_big,
# k_consensus_general<..> includes the k_decide pass that precedes it
KERNELS = ("k_recmeta<ss>", "k_consensus_fast<ss>", "k_consensus_exact<ss>", "k_consensus_general<ss>",
           "k_recmeta<ds>", "k_consensus_fast<ds>", "k_consensus_exact<ds>", "k_consensus_general<ds>")

_lib = None

# numpy view of dcr_read_info (include/dcr.h), 24 bytes
READ_INFO_DTYPE = np.dtype([("seq_start", "<i8"), ("len", "<i4"), ("n_cig", "<i4"), ("status", "<i4"),
                            ("has_ins", "<i4")])
assert READ_INFO_DTYPE.itemsize == ctypes.sizeof(DcrReadInfo)


class DcrError(RuntimeError):
    pass


def load():
    """Load libdcr.so (raises if absent: build it with __graft_entry__.build())."""
    global _lib
    if _lib is None:
        # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's):
        # load it first so libdcr and torch's allocator share one HIP runtime
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = os.environ.get("DCR_LIB_PATH", LIB_PATH)     # diagnostic builds (tools/)
        if not os.path.exists(path):
            raise DcrError(f"{path} not built — run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dcr_abi_version() != 1:
            raise DcrError("libdcr.so ABI mismatch")
        _lib = lib
    return _lib


def _check(rc):
    if rc != 0:
        raise DcrError(f"libdcr error {rc}: {load().dcr_last_error().decode()}")


class Context:
    """One GPU context (``dcr_ctx``): stream, parameters, workspace."""

    def __init__(self, params: ConsensusParams = ConsensusParams(), device: int = 0, want_info: bool = False):
        """``want_info``: write every read's preprocessing info (DCR_OPT_READ_INFO,
        parity tests); the product path only needs failing reads'."""
        lib = load()
        self.params = params
        self._p = build_dcr_params(params)
        self.device = device
        self._ctx = lib.dcr_create(device, ctypes.byref(self._p))
        if not self._ctx:
            raise DcrError(f"dcr_create failed: {lib.dcr_last_error().decode()}")
        self.want_info = want_info
        if want_info:
            _check(lib.dcr_set_options(self._ctx, 1))

    def close(self):
        if getattr(self, "_ctx", None):
            load().dcr_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, params: ConsensusParams):
        self.params = params
        self._p = build_dcr_params(params)
        _check(load().dcr_set_params(self._ctx, ctypes.byref(self._p)))

    @property
    def stream(self):
        return load().dcr_stream(self._ctx)

    # -- host-pointer path ------------------------------------------------
    def run_host(self, packed: PackedBatch, want_info=None):
        ss = OutArrays(4 * packed.n_fam, packed.ss_cols)
        ds = OutArrays(2 * packed.n_fam, packed.ds_cols)
        b = packed.as_struct()
        so, do = ss.as_struct(), ds.as_struct()
        _check(load().dcr_run_batch_host(self._ctx, ctypes.byref(b), ctypes.byref(so), ctypes.byref(do)))
        if want_info is None:
            want_info = self.want_info
        info = self.read_info(packed.n_reads) if want_info else None
        return ss, ds, info

    def read_info(self, n):
        arr = np.zeros(max(n, 1), dtype=READ_INFO_DTYPE)
        _check(load().dcr_read_info_host(self._ctx, arr.ctypes.data, n))
        return {k: arr[k][:n].copy() for k in READ_INFO_DTYPE.names}

    # -- device-pointer path (inputs resident in HBM) ----------------------
    def reserve(self, batch_struct: DcrBatch):
        _check(load().dcr_reserve(self._ctx, ctypes.byref(batch_struct)))

    def run_device(self, batch_struct: DcrBatch, ss: DcrOut, ds: DcrOut):
        """Asynchronous on the context stream."""
        _check(load().dcr_run_batch(self._ctx, ctypes.byref(batch_struct), ctypes.byref(ss), ctypes.byref(ds)))

    def sync(self):
        _check(load().dcr_sync(self._ctx))

    def last_timing(self):
        ms = (ctypes.c_float * 4)()
        _check(load().dcr_last_timing(self._ctx, ms))
        return dict(prep=ms[0], single_strand=ms[1], duplex=ms[2], total=ms[3])

    def last_kernel_timing(self):
        """Per-kernel ms of the last batch (HIP events between the launches)."""
        ms = (ctypes.c_float * len(KERNELS))()
        _check(load().dcr_last_kernel_timing(self._ctx, ms))
        return dict(zip(KERNELS, ms))


# include/dcr_inflate.h dcr_bgzf_member (32 bytes)
BGZF_MEMBER_DTYPE = np.dtype([("in_off", "<i8"), ("out_off", "<i8"), ("in_len", "<u4"), ("isize", "<u4"),
                              ("crc", "<u4"), ("pad", "<u4")])


class InflateHook(ctypes.Structure):
    """include/dcr_inflate.h dcr_inflate_hook (filled by dcr_inflater_hook)."""
    _fields_ = [("user", ctypes.c_void_p), ("run", ctypes.c_void_p), ("host_alloc", ctypes.c_void_p),
                ("host_free", ctypes.c_void_p), ("stream_open", ctypes.c_void_p), ("stream_add", ctypes.c_void_p),
                ("stream_fetch", ctypes.c_void_p), ("stream_close", ctypes.c_void_p)]


def bgzf_members(data) -> tuple:
    """(members, output bytes) of a buffer of whole BGZF blocks: the layout
    dcr_inflater_run takes (the ingest builds the same table natively)."""
    buf = memoryview(data)
    out, p, o = [], 0, 0
    while p < len(buf):
        if bytes(buf[p:p + 4]) != b"\x1f\x8b\x08\x04":
            raise ValueError(f"not a BGZF block at {p}")
        xlen = int.from_bytes(buf[p + 10:p + 12], "little")
        bsize, q = None, p + 12
        while q + 4 <= p + 12 + xlen:
            slen = int.from_bytes(buf[q + 2:q + 4], "little")
            if bytes(buf[q:q + 2]) == b"BC" and slen == 2:
                bsize = int.from_bytes(buf[q + 4:q + 6], "little") + 1
            q += 4 + slen
        if bsize is None:
            raise ValueError("BGZF block without BC field")
        crc = int.from_bytes(buf[p + bsize - 8:p + bsize - 4], "little")
        isize = int.from_bytes(buf[p + bsize - 4:p + bsize], "little")
        out.append((p + 12 + xlen, o, bsize - 12 - xlen - 8, isize, crc, 0))
        o += isize
        p += bsize
    return np.array(out, dtype=BGZF_MEMBER_DTYPE), o


class Inflater:
    """A device BGZF inflater (``dcr_inflater``, include/dcr_inflate.h)."""

    def __init__(self, device: int = 0):
        lib = load()
        self.device = device
        self._h = lib.dcr_inflater_create(device)
        if not self._h:
            raise DcrError(f"dcr_inflater_create failed: {lib.dcr_last_error().decode()}")

    @property
    def handle(self):
        return self._h

    def hook(self) -> InflateHook:
        h = InflateHook()
        _check(load().dcr_inflater_hook(self._h, ctypes.byref(h)))
        return h

    def run(self, data, members, out_bytes):
        """Inflate ``members`` of ``data`` (bytes / uint8 array): returns
        (0 or the index + 1 of the first failing member, output array)."""
        src = np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data
        m = np.ascontiguousarray(members, dtype=BGZF_MEMBER_DTYPE)
        out = np.zeros(max(out_bytes, 1), np.uint8)
        rc = load().dcr_inflater_run(self._h, src.ctypes.data, src.nbytes, m.ctypes.data, len(m), out.ctypes.data,
                                     out_bytes)
        if rc < 0:
            raise DcrError(f"dcr_inflater_run: {load().dcr_last_error().decode()}")
        return rc, out[:out_bytes]

    def last(self):
        ms, n = ctypes.c_float(), ctypes.c_int32()
        _check(load().dcr_inflater_last(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def totals(self, reset=False):
        """Kernel ms, runs, members and output bytes since creation / the last reset."""
        out = (ctypes.c_double * 4)()
        _check(load().dcr_inflater_totals(self._h, out, int(reset)))
        return {"kernel_ms": out[0], "runs": int(out[1]), "members": int(out[2]), "bytes": int(out[3])}

    def close(self):
        if getattr(self, "_h", None):
            load().dcr_inflater_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def backend(ctx: Context):
    """pipeline.Backend running on the GPU through the host-pointer entry."""
    def run(packed, params):
        if params != ctx.params:
            ctx.set_params(params)
        return ctx.run_host(packed)
    return run
