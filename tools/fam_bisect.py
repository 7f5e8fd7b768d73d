"""Diagnostic: which read of a C3 family's differing subfamily makes the HIP
path and the oracle disagree -- the family again with each read of that
subfamily left out in turn (one batch), plus minimal synthetic cases."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from duplexumiconsensusreads_amd import _lib, synth  # noqa: E402
from duplexumiconsensusreads_amd.batch import pack_families, subset_families  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams  # noqa: E402
from oracle import dcr_oracle_c  # noqa: E402


class Rd:
    def __init__(self, pos, mapq, seq, qual, cig):
        self.reference_start, self.mapping_quality = pos, mapq
        self.query_sequence, self.query_qualities, self.cigartuples = seq, qual, cig


def reads_of(s, r0, r1):
    out = []
    for i in range(r0, r1):
        o, L = int(s.seq_off[i]), int(s.seq_len[i])
        cig = [(int(c) & 15, int(c) >> 4) for c in s.cigar[s.cig_off[i]:s.cig_off[i] + s.cig_n[i]]]
        out.append(Rd(int(s.read_pos[i]), int(s.read_mapq[i]), bytes(s.bases[o:o + L]).decode(),
                      list(int(x) for x in s.quals[o:o + L]), cig))
    return out


def compare(fams, label, want_info=True):
    b = pack_families(fams)
    ctx = _lib.Context(ConsensusParams(), device=0, want_info=want_info)
    ss, ds, _ = ctx.run_host(b)
    sso, dso, _ = dcr_oracle_c.run(b, ConsensusParams())
    for k in range(len(fams)):
        ra, rb = ss.record(4 * k + 3, b.ss_col_off), sso.record(4 * k + 3, b.ss_col_off)
        same = all(np.array_equal(np.asarray(ra[x]), np.asarray(rb[x])) if hasattr(ra[x], "__len__") else ra[x] == rb[x]
                   for x in ra)
        if not same:
            da, db = list(ra["d"]), list(rb["d"])
            ks = [i for i in range(min(len(da), len(db))) if da[i] != db[i]]
            print(f"{label}[{k}] differs: d at {ks[:6]} gpu {[da[i] for i in ks[:6]]} cpu {[db[i] for i in ks[:6]]}",
                  flush=True)
        else:
            print(f"{label}[{k}] same", flush=True)


fam = int(sys.argv[1]) if len(sys.argv) > 1 else 34042
p = synth.packed_config(synth.CONFIGS["C3"], 400_000, seed=3)
s = subset_families(p, [fam])
subs = [reads_of(s, int(s.sub_off[k]), int(s.sub_off[k + 1])) for k in range(4)]
fams = [[subs[0], subs[1], subs[2], subs[3]]]
for v in range(len(subs[3])):
    fams.append([subs[0], subs[1], subs[2], subs[3][:v] + subs[3][v + 1:]])
compare(fams[:1], "no-info", want_info=False)
compare(fams[:1], "info", want_info=True)
compare(fams[:1] * 2, "twice")
compare(fams, "leave-one-out")
for v in range(len(fams)):                 # each variant alone in its batch
    compare(fams[v:v + 1], f"alone{v}")
# minimal cases: n full reads + one read with an insertion whose last base is masked
full = [r for r in subs[3] if r.cigartuples == [(0, 150)]][:4]
ins = [r for r in subs[3] if any(op == 1 for op, _ in r.cigartuples)]
clip = [r for r in subs[3] if any(op == 4 for op, _ in r.cigartuples)]
cases = [[subs[0], subs[1], subs[2], full + ins], [subs[0], subs[1], subs[2], full + clip],
         [subs[0], subs[1], subs[2], full + ins + clip], [subs[0], subs[1], subs[2], ins + clip]]
compare(cases, "minimal")
for r in ins + clip:
    print("read", r.reference_start, r.cigartuples, r.query_sequence[-4:], r.query_qualities[-4:],
          r.query_sequence[:4], r.query_qualities[:4], flush=True)
