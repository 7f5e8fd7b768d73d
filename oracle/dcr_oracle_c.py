"""ORACLE — test infrastructure only.  ctypes access to the C restatement
(oracle/dcr_oracle.c -> oracle/_build/libdcr_oracle.so), with the same
backend signature as the HIP runner so tests can compare them."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from duplexumiconsensusreads_amd.batch import DcrReadInfo, OutArrays
from duplexumiconsensusreads_amd.params import build_dcr_params

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libdcr_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.dcr_oracle_run.restype = ctypes.c_int
        _lib.dcr_oracle_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    return _lib


INFO_DTYPE = np.dtype([("seq_start", "<i8"), ("len", "<i4"), ("n_cig", "<i4"), ("status", "<i4"),
                       ("has_ins", "<i4")])
assert INFO_DTYPE.itemsize == ctypes.sizeof(DcrReadInfo)


def run(packed, params, n_threads=1, want_info=True):
    """Backend: returns (ss OutArrays, ds OutArrays, read-info dict)."""
    lib = load()
    P = build_dcr_params(params)
    ss = OutArrays(4 * packed.n_fam, packed.ss_cols)
    ds = OutArrays(2 * packed.n_fam, packed.ds_cols)
    info = np.zeros(max(packed.n_reads, 1), dtype=INFO_DTYPE)
    b = packed.as_struct()
    so, do = ss.as_struct(), ds.as_struct()
    rc = lib.dcr_oracle_run(ctypes.byref(P), ctypes.byref(b), ctypes.byref(so),
                            ctypes.byref(do), ctypes.c_void_p(info.ctypes.data), n_threads)
    if rc != 0:
        raise RuntimeError(f"dcr_oracle_run failed: {rc}")
    n = packed.n_reads
    return ss, ds, ({k: info[k][:n].copy() for k in INFO_DTYPE.names} if want_info else None)
