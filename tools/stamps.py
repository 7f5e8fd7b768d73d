"""Diagnostic: per-phase s_memtime cycle totals of the fast consensus kernel
(a DCR_STAMP=1 build of libdcr: tools/build_variant.sh stamp "-DDCR_STAMP=1") on the C2 batch.
usage: python tools/stamps.py FAMILIES LIB"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from duplexumiconsensusreads_amd import synth  # noqa: E402
from duplexumiconsensusreads_amd.device import DeviceBatch  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams, build_dcr_params  # noqa: E402

nfam, path = int(sys.argv[1]), sys.argv[2]
cfg = os.environ.get("ABL_CONFIG", "C2")
packed = (synth.packed_fixed_size(nfam, seed=3) if cfg == "C2"
          else synth.packed_config(synth.CONFIGS[cfg], nfam, seed=3, max_reads=1000))
db = DeviceBatch(packed)
P = build_dcr_params(ConsensusParams())
lib = ctypes.CDLL(path)
lib.dcr_create.restype = ctypes.c_void_p
lib.dcr_create.argtypes = [ctypes.c_int, ctypes.c_void_p]
for n in ("dcr_run_batch", "dcr_sync", "dcr_last_kernel_timing", "dcr_debug_stamps"):
    getattr(lib, n).restype = ctypes.c_int
lib.dcr_run_batch.argtypes = [ctypes.c_void_p] * 4
lib.dcr_sync.argtypes = [ctypes.c_void_p]
lib.dcr_last_kernel_timing.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
lib.dcr_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
ctx = lib.dcr_create(0, ctypes.byref(P))
st = (ctypes.c_ulonglong * 64)()
run = lambda: lib.dcr_run_batch(ctx, ctypes.byref(db.batch_struct), ctypes.byref(db.ss_struct), ctypes.byref(db.ds_struct))
assert run() == 0 and lib.dcr_sync(ctx) in (0, 3)
lib.dcr_debug_stamps(ctx, st, 64, 1)
K = 3
kt = [0.0] * 7
for _ in range(K):
    assert run() == 0
    ms = (ctypes.c_float * 9)()
    lib.dcr_last_kernel_timing(ctx, ms)
    kt = [a + b for a, b in zip(kt, ms)]
lib.dcr_debug_stamps(ctx, st, 64, 0)
names = ["prefetch wait", "codes into LDS", "prefetch issue", "trim, fence", "products",
         "finalize: rest", "depth reductions", "column stores", "mean", "record scalars",
         "finalize: exact cols", "finalize: decision"]
for kind, base, nrec, kidx in (("single-strand fast", 0, 4 * nfam, 1), ("duplex fast", 16, 2 * nfam, 5),
                               ("single-strand exact", 32, 4 * nfam, 2), ("duplex exact", 48, 2 * nfam, 6)):
    tot = sum(st[base + k] for k in range(12))
    print(f"{kind}: kernel {kt[kidx] / K:.3f} ms; cycles per record per wave (s_memtime ticks):")
    for k in range(12):
        print(f"   {names[k]:18s} {st[base + k] / (K * nrec):10.1f}  ({100.0 * st[base + k] / max(tot, 1):5.1f} %)")
