"""Diagnostic: per-phase s_memtime cycle totals of the general consensus kernel
(a DCR_GSTAMP=1 build of libdcr: tools/build_variant.sh gstamp "-DDCR_GSTAMP=1")
on one HBM-resident batch of a config (ABL_CONFIG, default C3), with the
cycles and counts per record class.
usage: python tools/gstamps.py FAMILIES LIB"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from duplexumiconsensusreads_amd import synth  # noqa: E402
from duplexumiconsensusreads_amd.device import DeviceBatch  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams, build_dcr_params  # noqa: E402

nfam, path = int(sys.argv[1]), sys.argv[2]
cfg = os.environ.get("ABL_CONFIG", "C3")
packed = synth.packed_config(synth.CONFIGS[cfg], nfam, seed=3, max_reads=1000)
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
kt = [0.0] * 8
for _ in range(K):
    assert run() == 0
    ms = (ctypes.c_float * 9)()
    lib.dcr_last_kernel_timing(ctx, ms)
    kt = [a + b for a, b in zip(kt, ms)]
lib.dcr_debug_stamps(ctx, st, 64, 0)
phases = ["setup", "codes + flag pass", "window loads", "layout steps", "decide / products",
          "finalize + d/e", "adjust (phase 3)", "mean + scalars"]
classes = ["no insertion", "insertion, <= 64 reads", "insertion, 65-256 reads (registers)", "insertion, other"]
for kind, base, kidx in (("single-strand", 0, 3), ("duplex", 32, 7)):
    tot = sum(st[base + k] for k in range(8))
    nrec = sum(st[base + 12 + c] for c in range(4)) / K
    print(f"{kind} general: kernel {kt[kidx] / K:.3f} ms, {nrec:.0f} records; s_memtime ticks per record per wave:")
    for k in range(8):
        print(f"   {phases[k]:22s} {st[base + k] / max(K * nrec, 1):10.1f}  ({100.0 * st[base + k] / max(tot, 1):5.1f} %)")
    if st[base + 16]:
        print(f"   small insertion layouts: {st[base + 16] / K:.0f} column steps, drain before the steps "
              f"{st[base + 17] / max(st[base + 16], 1):.1f} ticks per step")
    for c in range(4):
        n = st[base + 12 + c] / K
        cyc = st[base + 8 + c] / K
        print(f"   class {classes[c]:38s} records {n:9.0f}  ticks/record {cyc / max(n, 1):10.1f}  share {100.0 * cyc / max(sum(st[base + 8 + j] for j in range(4)) / K, 1):5.1f} %")
lcls = ["not laid out (no insertion, ineligible)", "laid out, <= 64 reads", "laid out, 65-256 reads"]
print(f"k_ins_layout<ss>: s_memtime ticks per record per wave (its slot is inside the general slot above); "
      f"longest record {st[26]} ticks")
for c in range(3):
    n = st[23 + c] / K
    print(f"   {lcls[c]:42s} records {n:9.0f}  ticks/record {st[20 + c] / K / max(n, 1):10.1f}")
