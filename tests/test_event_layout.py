"""The general kernel's insertion layout by events (csrc/dcr_kernels.hip,
EvLds / ev_next / the ev_ok tile branch) restated step for step in Python and
checked against the oracle's column-by-column reconstruct_alignment
(oracle/dcr_oracle.py reconstruct, reference :430-547) on random reads: I and
D runs anywhere (leading I before a read's start, I at the sequence's end,
several I runs per read), reads starting inside insertion blocks, CIGARs
whose ops do not match the sequence length (the 3'-trim quirk, :320-323) with
their IndexErrors, and =/X/N/P ops."""
import random

import pytest

from oracle import dcr_oracle

BIG = 0x7FFFFFFF


def ev_next(cig, ln_seq, k, md, sq):
    """(k, m, L, s0) of the next reachable I run from run k, or None."""
    for kk in range(k, len(cig)):
        op, ln = cig[kk]
        if op == 1:
            return (kk, md, ln, sq)
        if sq >= ln_seq:
            return None
        if op != 2 and sq + ln > ln_seq:
            return None
        md += ln
        if op != 2:
            sq += ln
    return None


def event_layout(pos, cigs, seqs):
    """Blocks and per-column elements exactly as the kernel derives them:
    returns (rows of (kind, seq index) per read, index_error)."""
    R = len(pos)
    minpos = min(pos)
    T = max(p + len(s) for p, s in zip(pos, seqs)) - minpos
    lens = [len(s) for s in seqs]
    ev = []
    for r in range(R):
        nx = ev_next(cigs[r], lens[r], 0, 0, 0)
        ev.append({"s": pos[r] - minpos, "A": 0, "nx": nx})
    blocks = []          # (start, len, {read: (s0, L)})
    t = 0
    while True:
        tr = []
        for e in ev:
            if e["nx"] is None:
                tr.append(BIG)
                continue
            _, m, _, _ = e["nx"]
            tr.append(t if m == e["A"] else max(t, e["s"]) + (m - e["A"]))
        te = min(tr)
        if te >= T:
            break
        part = {}
        lmax = 0
        for r, e in enumerate(ev):
            e["A"] += max(0, te - max(t, e["s"]))
            if tr[r] == te:
                k, m, L, s0 = e["nx"]
                part[r] = (s0, L)
                lmax = max(lmax, L)
                e["nx"] = ev_next(cigs[r], lens[r], k + 1, m, s0 + L)
        blocks.append((te, min(lmax, T - te), part))
        t = te + lmax
    ns = []
    for e in ev:
        ib = sum(min(max(e["s"] - b, 0), bl) for b, bl, _ in blocks)
        ns.append(e["s"] - ib)
    rows = [[] for _ in range(R)]
    err = False
    for tcol in range(T):
        insb, bi, bo = 0, None, 0
        for b, (bs, bl, _) in enumerate(blocks):
            if tcol >= bs + bl:
                insb += bl
            elif tcol >= bs:
                bi, bo = b, tcol - bs
        nt = tcol - insb
        for r in range(R):
            if bi is not None:
                part = blocks[bi][2]
                if r not in part or bo >= part[r][1]:
                    rows[r].append(("+", None))
                    continue
                is_ = part[r][0] + bo
                if is_ >= lens[r]:
                    err = True
                    rows[r].append(("N", None))
                    continue
                rows[r].append(("ins", is_))
                continue
            av = nt - ns[r]
            if av < 0:
                rows[r].append(("N", None))
                continue
            acc = sq = 0
            out = None
            for op, ln in cigs[r]:
                if op == 1:
                    sq += ln
                    continue
                if av < acc + ln:
                    is_ = sq + (av - acc if op != 2 else 0)
                    out = ("N", None) if is_ >= lens[r] else (("-", None) if op == 2 else ("M", is_))
                    break
                acc += ln
                if op != 2:
                    sq += ln
            if out is None:
                if sq < lens[r]:
                    err = True
                out = ("N", None)
            rows[r].append(out)
    return rows, err


def as_chars(rows, seqs):
    out = []
    for r, row in enumerate(rows):
        line = []
        for kind, is_ in row:
            if kind == "ins":
                line.append(seqs[r][is_].lower())
            elif kind == "M":
                line.append(seqs[r][is_])
            else:
                line.append(kind)
        out.append(line)
    return out


def rand_case(rng, consistent=True):
    R = rng.randint(1, 12)
    pos, cigs, seqs = [], [], []
    for _ in range(R):
        runs = []
        for _ in range(rng.randint(1, 5)):
            op = rng.choice([0, 0, 0, 1, 1, 2, 2, 7, 8, 3])
            runs.append((op, rng.randint(1, 6)))
        # merge equal neighbours as the normalised runs are
        norm = []
        for op, ln in runs:
            o = 0 if op in (7, 8) else op
            if norm and norm[-1][0] == o:
                norm[-1] = (o, norm[-1][1] + ln)
            else:
                norm.append((o, ln))
        consume = sum(ln for op, ln in norm if op != 2)
        if consistent:
            n = consume
        else:
            n = max(1, consume + rng.randint(-3, 3))
        if n == 0:
            norm.append((0, 1))
            n = 1
        pos.append(rng.randint(0, 8))
        cigs.append(norm)
        seqs.append("".join(rng.choice("ACGTN") for _ in range(n)))
    return pos, cigs, seqs


@pytest.mark.parametrize("consistent", [True, False])
def test_event_layout_equals_column_by_column(consistent):
    rng = random.Random(7 if consistent else 8)
    n_err = n_ins = 0
    for case in range(4000):
        pos, cigs, seqs = rand_case(rng, consistent)
        rows, err = event_layout(pos, cigs, seqs)
        try:
            al, _, _ = dcr_oracle.reconstruct(pos, cigs, seqs, [[30] * len(s) for s in seqs])
            ref_err = False
        except dcr_oracle.RefCrash as e:
            assert e.kind == "IndexError"
            ref_err = True
        assert err == ref_err, (case, pos, cigs, seqs)
        if ref_err:
            n_err += 1
            continue
        got = as_chars(rows, seqs)
        assert got == al, (case, pos, cigs, seqs)
        n_ins += any("+" in row for row in al)
    assert n_ins > 300
    if not consistent:
        assert n_err > 100
