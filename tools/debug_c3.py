"""Debug: locate the differing columns of failing records of the C3-shape parity case."""
import sys
import numpy as np
sys.path.insert(0, ".")
from duplexumiconsensusreads_amd import _lib, synth
from duplexumiconsensusreads_amd.params import ConsensusParams
from oracle import dcr_oracle_c

packed = synth.packed_config(synth.CONFIGS["C3"], 3000, seed=21, max_reads=1000)
params = ConsensusParams(max_reads=1000)
ctx = _lib.Context(params, device=0)
g = ctx.run_host(packed)
w = dcr_oracle_c.run(packed, params, n_threads=8)
nbad = 0
for kind, col_off, a, b in (("ss", packed.ss_col_off, g[0], w[0]), ("ds", packed.ds_col_off, g[1], w[1])):
    for i in range(a.n_rec):
        if a.status[i] != 0:
            continue
        ra, rb = a.record(i, col_off), b.record(i, col_off)
        if ra == rb:
            continue
        nbad += 1
        if nbad > 6:
            continue
        print("==", kind, i, "keys differing:", [k for k in ra if ra[k] != rb[k]])
        for k in ra:
            if ra[k] != rb[k] and isinstance(ra[k], (list, str, bytes)):
                x, y = list(ra[k]), list(rb[k])
                idx = [j for j in range(max(len(x), len(y))) if j >= len(x) or j >= len(y) or x[j] != y[j]]
                print("  ", k, "len", len(x), len(y), "idx", idx[:20])
                print("   got ", [x[j] for j in idx[:20] if j < len(x)])
                print("   want", [y[j] for j in idx[:20] if j < len(y)])
        if kind == "ss":
            a0, a1 = packed.sub_off[i], packed.sub_off[i + 1]
            print("   R", a1 - a0, "T", ra.get("len"), "pos", ra.get("pos"))
            for r in range(a0, a1):
                c = packed.cigar[packed.cig_off[r]:packed.cig_off[r] + packed.cig_n[r]]
                if packed.cig_n[r] > 1:
                    print("    read", r - a0, "pos", packed.read_pos[r], [(int(v >> 4), "MIDNSHP=X"[v & 15]) for v in c])
print("records differing:", nbad)
