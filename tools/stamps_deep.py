"""Diagnostic: per-phase s_memtime cycle totals of k_decide_deep (a
DCR_STAMP=1 build of libdcr) on a C4-shape batch.
usage: python tools/stamps_deep.py FAMILIES LIB"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from duplexumiconsensusreads_amd import synth  # noqa: E402
from duplexumiconsensusreads_amd.device import DeviceBatch  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams, build_dcr_params  # noqa: E402

nfam, path = int(sys.argv[1]), sys.argv[2]
packed = synth.packed_config(synth.CONFIGS["C4"], n_families=nfam, max_reads=1000)
db = DeviceBatch(packed)
P = build_dcr_params(ConsensusParams(max_reads=1000))
lib = ctypes.CDLL(path)
lib.dcr_create.restype = ctypes.c_void_p
lib.dcr_create.argtypes = [ctypes.c_int, ctypes.c_void_p]
for n in ("dcr_run_batch", "dcr_sync", "dcr_debug_stamps"):
    getattr(lib, n).restype = ctypes.c_int
lib.dcr_run_batch.argtypes = [ctypes.c_void_p] * 4
lib.dcr_sync.argtypes = [ctypes.c_void_p]
lib.dcr_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
ctx = lib.dcr_create(0, ctypes.byref(P))
st = (ctypes.c_ulonglong * 32)()
run = lambda: lib.dcr_run_batch(ctx, ctypes.byref(db.batch_struct), ctypes.byref(db.ss_struct), ctypes.byref(db.ds_struct))
assert run() == 0 and lib.dcr_sync(ctx) in (0, 3)
lib.dcr_debug_stamps(ctx, st, 32, 1)
K = 3
for _ in range(K):
    assert run() == 0
assert lib.dcr_sync(ctx) in (0, 3)
lib.dcr_debug_stamps(ctx, st, 32, 0)
nrec = 4 * nfam
names = ["checks over the reads", "the wave's rows", "decision + barriers"]
tot = sum(st[26 + k] for k in range(3))
print(f"k_decide_deep: cycles per record per wave (s_memtime ticks), {packed.n_reads} reads, {nrec} records")
for k in range(3):
    print(f"   {names[k]:24s} {st[26 + k] / (K * nrec):10.1f}  ({100.0 * st[26 + k] / max(tot, 1):5.1f} %)")
