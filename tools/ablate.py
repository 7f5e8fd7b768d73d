"""Diagnostic: time the kernels of several libdcr builds (ablation variants
built with -DDCR_ABL=n, or candidate kernels) on one HBM-resident batch,
interleaved in one process.  After each build's first run its outputs (every
single-strand and duplex array) are hashed: a build whose digest differs from
the first build's is marked DIFFERS (ablation builds are expected to differ;
candidate kernels are not)."""
import hashlib
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from duplexumiconsensusreads_amd import synth  # noqa: E402
from duplexumiconsensusreads_amd.device import DeviceBatch  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams, build_dcr_params  # noqa: E402

libs = sys.argv[2:]
nfam = int(sys.argv[1])
cfg = os.environ.get("ABL_CONFIG", "C2")
packed = (synth.packed_fixed_size(nfam, seed=3) if cfg == "C2"
          else synth.packed_config(synth.CONFIGS[cfg], nfam, seed=3, max_reads=1000))
if os.environ.get("ABL_SS_ALIGN"):
    # diagnostic: single-strand output regions rounded up to ABL_SS_ALIGN
    # columns instead of 16 (the kernels still write T16 columns of each)
    import numpy as np
    al = int(os.environ["ABL_SS_ALIGN"])
    t = np.diff(packed.ss_col_off)
    t = (t + al - 1) // al * al
    packed.ss_col_off[1:] = np.cumsum(t)
db = DeviceBatch(packed)
P = build_dcr_params(ConsensusParams())
handles = []
for path in libs:
    lib = ctypes.CDLL(path)
    lib.dcr_create.restype = ctypes.c_void_p
    lib.dcr_create.argtypes = [ctypes.c_int, ctypes.c_void_p]
    for n in ("dcr_run_batch", "dcr_sync", "dcr_last_timing", "dcr_last_kernel_timing"):
        getattr(lib, n).restype = ctypes.c_int
    lib.dcr_run_batch.argtypes = [ctypes.c_void_p] * 4
    lib.dcr_sync.argtypes = [ctypes.c_void_p]
    lib.dcr_last_timing.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.dcr_last_kernel_timing.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ctx = lib.dcr_create(0, ctypes.byref(P))
    handles.append((path, lib, ctx))
res = {p: [] for p in libs}
digest = {}


def _ranges(off, n):
    """indices of [off_i, off_i + n_i) for every record, concatenated"""
    import numpy as np
    n = np.maximum(n.astype(np.int64), 0)
    tot = int(n.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    start = np.repeat(off.astype(np.int64) - (np.cumsum(n) - n), n)
    return np.arange(tot, dtype=np.int64) + start


def out_digest():
    """sha1 over every record's scalars and its defined columns only (seq /
    qual over len, CIGAR over n_cig, d / e over n_de; nothing of a failed
    record): region tails are don't-care and may hold stale words"""
    import numpy as np
    import torch
    torch.cuda.synchronize()
    h = hashlib.sha1()
    ss, ds = db.download()
    for oa, col_off in ((ss, packed.ss_col_off), (ds, packed.ds_col_off)):
        ok = oa.status == 0
        for k in ("status", "pos", "mapq", "len", "n_cig", "n_de", "D", "M", "E"):
            h.update(np.ascontiguousarray(getattr(oa, k)).tobytes())
        off = np.asarray(col_off[:-1])
        for k, n in (("seq", oa.len), ("qual", oa.len), ("cigar", oa.n_cig), ("d", oa.n_de), ("e", oa.n_de)):
            h.update(getattr(oa, k)[_ranges(off, np.where(ok, n, 0))].tobytes())
    return h.hexdigest()[:12]


for rnd in range(6):
    for path, lib, ctx in handles:
        assert lib.dcr_run_batch(ctx, ctypes.byref(db.batch_struct), ctypes.byref(db.ss_struct),
                                 ctypes.byref(db.ds_struct)) == 0
        rc = lib.dcr_sync(ctx)
        assert rc in (0, 3), (path, rnd, rc)
        ms = (ctypes.c_float * 9)()
        lib.dcr_last_kernel_timing(ctx, ms)
        if rnd:
            res[path].append(list(ms))
        else:
            digest[path] = out_digest()
            for kind in ("ss", "ds"):
                for v in db.out[kind].values():
                    v.zero_()
for path, lib, ctx in handles:
    if hasattr(lib, "dcr_debug_counts"):
        c = (ctypes.c_int * 10)()
        lib.dcr_debug_counts(ctypes.c_void_p(ctx), c)
        print(f"{os.path.basename(path):24s} counts: fast ss/ds {c[3]}/{c[4]} exact ss/ds {c[5]}/{c[6]} "
              f"ovf {c[1]}/{c[2]} deep {c[9]}")
        break
for path in libs:
    v = res[path]
    med = [sorted(x[k] for x in v)[len(v) // 2] for k in range(9)]
    same = "same" if digest[path] == digest[libs[0]] else "DIFFERS"
    print(f"{os.path.basename(path):24s} slots(ms): " + " ".join(f"{m:7.3f}" for m in med) + f"  sum {sum(med):7.3f}"
          f"  out {digest[path]} {same}")
