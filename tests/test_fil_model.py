"""The insertion layout by events (tests/fil_model.py) against the oracle's
column-by-column reconstruct_alignment (DuplexUMIConsensusReads.py:430-547) on
random subfamilies with insertions, deletions, soft clips, leading insertions,
late-starting reads and trimmed 3' N tails."""
import random

import pytest

from oracle import dcr_oracle as O
from tests.fil_model import fil_layout


def _read(rng, L):
    bases = "".join(rng.choice("ACGT") for _ in range(L))
    quals = [rng.choice([37, 37, 37, 25, 12, 2]) for _ in range(L)]
    if rng.random() < 0.15:                       # sequenced N tail (3' trim)
        k = rng.randint(1, 6)
        bases = bases[:-k] + "N" * k
    ops = []
    body = L
    s5 = s3 = 0
    if rng.random() < 0.1:
        s5 = rng.randint(1, 8)
    if rng.random() < 0.1:
        s3 = rng.randint(1, 8)
    body = L - s5 - s3
    kind = rng.random()
    if kind < 0.35 and body > 10:                  # one insertion
        a = rng.randint(0, body - 4) if rng.random() < 0.9 else 0
        li = rng.randint(1, 3)
        li = min(li, body - a)
        ops = [(0, a), (1, li), (0, body - a - li)]
    elif kind < 0.5 and body > 10:                 # one deletion
        a = rng.randint(1, body - 2)
        ops = [(0, a), (2, rng.randint(1, 3)), (0, body - a)]
    elif kind < 0.55 and body > 12:                # insertion and deletion
        a = rng.randint(1, body // 2 - 2)
        li = rng.randint(1, 2)
        ops = [(0, a), (1, li), (0, 3), (2, 2), (0, body - a - li - 3)]
    else:
        ops = [(0, body)]
    ops = [(o, n) for o, n in ops if n > 0]
    cig = ([(4, s5)] if s5 else []) + ops + ([(4, s3)] if s3 else [])
    return cig, bases, quals


def _family(rng):
    R = rng.choice([1, 2, 3, 5, 8, 13, 20, 40])
    base = 1000
    L = rng.choice([20, 40, 75, 150])
    reads = []
    for _ in range(R):
        cig, b, q = _read(rng, L)
        reads.append((base + rng.randint(0, 12), cig, b, q))
    return reads


@pytest.mark.parametrize("seed", range(6))
def test_fil_layout_matches_reconstruct(seed):
    rng = random.Random(seed)
    checked = skipped = crashed = 0
    for _ in range(400):
        fam = _family(rng)
        pos, cigs, seqs, quals = [], [], [], []
        try:
            for p, cig, b, q in fam:
                c2, s2, q2 = O.preprocess_read(cig, b, q, 20)
                pos.append(p)
                cigs.append(c2)
                seqs.append(s2)
                quals.append(q2)
        except O.RefCrash:
            continue
        try:
            ref = O.reconstruct(pos, cigs, seqs, quals)
        except O.RefCrash:
            ref = None
        got = fil_layout(pos, cigs, seqs, quals)
        if got is None:
            skipped += 1
            continue
        assert ref is not None, "the model laid out a record the reference raises on"
        assert got[2] == ref[2]
        assert got[0] == ref[0] and got[1] == ref[1]
        checked += 1
        crashed += ref is None
    assert checked > 200 and skipped < checked
