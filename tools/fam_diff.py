"""Diagnostic: one C3 family (synth.packed_config(C3, 400k, seed 3)) through
the HIP path alone and inside its neighbours, against the C oracle: the
single-strand / duplex records whose columns differ, column by column."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from duplexumiconsensusreads_amd import _lib, synth  # noqa: E402
from duplexumiconsensusreads_amd.batch import subset_families  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams  # noqa: E402
from oracle import dcr_oracle_c  # noqa: E402

fam = int(sys.argv[1]) if len(sys.argv) > 1 else 34042
p = synth.packed_config(synth.CONFIGS["C3"], 400_000, seed=3)
params = ConsensusParams()
ctx = _lib.Context(params, device=0, want_info=True)
for lo, hi in ((fam, fam + 1), (fam - 64, fam + 64), (fam - 4096, fam + 4096)):
    s = subset_families(p, list(range(lo, hi)))
    ss, ds, info = ctx.run_host(s)
    sso, dso, infoo = dcr_oracle_c.run(s, params)
    k = fam - lo
    print(f"== families [{lo}, {hi}): target index {k}", flush=True)
    for name, a, b, off, n in (("ss", ss, sso, s.ss_col_off, 4), ("ds", ds, dso, s.ds_col_off, 2)):
        for j in range(n):
            ra, rb = a.record(n * k + j, off), b.record(n * k + j, off)
            if ra == rb:
                continue
            print(f"  {name}[{j}] differs:", flush=True)
            for key in ra:
                va, vb = ra[key], rb[key]
                if isinstance(va, np.ndarray) or isinstance(va, list):
                    va, vb = list(va), list(vb)
                if va != vb:
                    if isinstance(va, list):
                        ks = [i for i in range(min(len(va), len(vb))) if va[i] != vb[i]]
                        print(f"    {key}: len {len(va)}/{len(vb)} differ at {ks[:10]}: "
                              f"gpu {[va[i] for i in ks[:10]]} cpu {[vb[i] for i in ks[:10]]}", flush=True)
                    else:
                        print(f"    {key}: gpu {va} cpu {vb}", flush=True)
    r0, r1 = int(s.sub_off[4 * k]), int(s.sub_off[4 * k + 4])
    print("  read info gpu:", [tuple(int(x) for x in info[i].tolist()) if hasattr(info[i], 'tolist') else info[i]
                                for i in range(r0, r1)][:40], flush=True)
